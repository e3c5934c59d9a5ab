// HAVAL and Lyra2 (see legacy_algos.hpp for the reference call sites).
//
// HAVAL: the eight IV words and the 128 round constants of passes 2-5 are consecutive 32-bit words
// of pi's fractional part (IV = words 0-7, pass p uses words 8+32(p-2) ..), so they are computed
// here with the BBP digit-extraction formula instead of being tabulated; a start-up check pins the
// first IV word and the first pass-2 constant. The reference unrolls every (passes, pass) pair into
// its own macro (haval.c:123-223); here one step routine takes the pass's phi permutation and word
// order as data and rotates the 8-word state by index.
#include "legacy_algos.hpp"

#include <cmath>
#include <cstring>
#include <stdexcept>

namespace nodexa {

namespace {

// ------------------------------------------------------------------ pi words (BBP)

u64 pow16_mod(u64 e, u64 m) {
    u64 r = 1 % m, b = 16 % m;
    while (e) {
        if (e & 1) r = r * b % m;
        b = b * b % m;
        e >>= 1;
    }
    return r;
}

// frac(sum_k 16^(n-k) / (8k+j))
double bbp_series(int j, u64 n) {
    double s = 0.0;
    for (u64 k = 0; k <= n; ++k) {
        const u64 d = 8 * k + u64(j);
        s += double(pow16_mod(n - k, d)) / double(d);
        s -= std::floor(s);
    }
    double p = 1.0 / 16.0;
    for (u64 k = n + 1; k < n + 24; ++k, p /= 16.0) s += p / double(8 * k + u64(j));
    return s - std::floor(s);
}

// four hex digits of pi's fraction starting after position n (digits n+1..n+4)
u32 pi_hex4(u64 n) {
    double x = 4 * bbp_series(1, n) - 2 * bbp_series(4, n) - bbp_series(5, n) - bbp_series(6, n);
    x -= std::floor(x);
    return u32(x * 65536.0) & 0xffffu;
}

struct PiWords {
    u32 w[136];
    PiWords() {
        for (int i = 0; i < 136; ++i) w[i] = (pi_hex4(u64(8 * i)) << 16) | pi_hex4(u64(8 * i + 4));
        if (w[0] != 0x243F6A88u || w[8] != 0x452821E6u) throw std::logic_error("HAVAL constants");
    }
};

const PiWords& pi_words() {
    static const PiWords p;
    return p;
}

// ------------------------------------------------------------------ HAVAL

inline u32 rotr(u32 x, int n) { return (x >> n) | (x << (32 - n)); }
inline u32 rotl(u32 x, int n) { return n ? (x << n) | (x >> (32 - n)) : x; }

// Boolean functions of the paper, arguments in the order (x6, x5, x4, x3, x2, x1, x0).
u32 haval_f(int f, const u32 a[7]) {
    const u32 x6 = a[0], x5 = a[1], x4 = a[2], x3 = a[3], x2 = a[4], x1 = a[5], x0 = a[6];
    switch (f) {
        case 1: return (x1 & x4) ^ (x2 & x5) ^ (x3 & x6) ^ (x0 & x1) ^ x0;
        case 2:
            return (x1 & x2 & x3) ^ (x2 & x4 & x5) ^ (x1 & x2) ^ (x1 & x4) ^ (x2 & x6) ^ (x3 & x5) ^ (x4 & x5) ^
                   (x0 & x2) ^ x0;
        case 3: return (x1 & x2 & x3) ^ (x1 & x4) ^ (x2 & x5) ^ (x3 & x6) ^ (x0 & x3) ^ x0;
        case 4:
            return (x1 & x2 & x3) ^ (x2 & x4 & x5) ^ (x3 & x4 & x6) ^ (x1 & x4) ^ (x2 & x6) ^ (x3 & x4) ^
                   (x3 & x5) ^ (x3 & x6) ^ (x4 & x5) ^ (x4 & x6) ^ (x0 & x4) ^ x0;
        default: return (x1 & x4) ^ (x2 & x5) ^ (x3 & x6) ^ (x0 & x1 & x2 & x3) ^ (x0 & x5) ^ x0;
    }
}

// phi_{n,p}: which x_i feeds each of F_p's (x6..x0) slots, for n passes.
const u8 kPhi[3][5][7] = {
    {{1, 0, 3, 5, 6, 2, 4}, {4, 2, 1, 0, 5, 3, 6}, {6, 1, 2, 3, 4, 5, 0}},
    {{2, 6, 1, 4, 5, 3, 0}, {3, 5, 2, 0, 1, 6, 4}, {1, 4, 3, 6, 0, 2, 5}, {6, 4, 0, 5, 2, 1, 3}},
    {{3, 4, 1, 0, 5, 2, 6}, {6, 2, 1, 0, 3, 4, 5}, {2, 6, 0, 4, 3, 1, 5}, {1, 5, 3, 2, 0, 4, 6}, {2, 5, 0, 6, 4, 3, 1}},
};

// Message-word order of passes 2-5 (pass 1 reads the words in order).
const u8 kOrder[4][32] = {
    {5, 14, 26, 18, 11, 28, 7, 16, 0, 23, 20, 22, 1, 10, 4, 8, 30, 3, 21, 9, 17, 24, 29, 6, 19, 12, 15, 13, 2, 25, 31, 27},
    {19, 9, 4, 20, 28, 17, 8, 22, 29, 14, 25, 12, 24, 30, 16, 26, 31, 15, 7, 3, 1, 0, 18, 27, 13, 6, 21, 10, 23, 11, 5, 2},
    {24, 4, 0, 14, 2, 7, 28, 23, 26, 6, 30, 20, 18, 25, 19, 3, 22, 11, 31, 21, 8, 27, 12, 9, 1, 29, 5, 15, 17, 10, 16, 13},
    {27, 3, 21, 26, 17, 11, 20, 29, 19, 0, 12, 7, 13, 8, 31, 10, 5, 9, 14, 30, 18, 6, 28, 24, 2, 23, 16, 22, 4, 1, 25, 15},
};

void haval_block(u32 s[8], const u8* blk, int passes) {
    u32 w[32];
    for (int i = 0; i < 32; ++i) w[i] = load_le32(blk + 4 * i);
    const u32* pi = pi_words().w;
    u32 v[8];
    std::memcpy(v, s, sizeof v);
    for (int p = 1; p <= passes; ++p) {
        const u8* phi = kPhi[passes - 3][p - 1];
        for (int i = 0; i < 32; ++i) {
            // step i writes x7 = v[(7 - i) mod 8]; x_k is v[(k - i) mod 8]
            const int j = i & 7;
            u32 a[7];
            for (int k = 0; k < 7; ++k) a[k] = v[(phi[k] - j) & 7];
            const u32 t = haval_f(p, a);
            u32& x7 = v[(7 - j) & 7];
            const u32 word = p == 1 ? w[i] : w[kOrder[p - 2][i]];
            const u32 c = p == 1 ? 0u : pi[8 + 32 * (p - 2) + i];
            x7 = rotr(t, 7) + rotr(x7, 11) + word + c;
        }
    }
    for (int i = 0; i < 8; ++i) s[i] += v[i];
}

// Output tailoring of the paper (folding s[5..7] / s[4..7] into shorter digests).
void haval_fold(const u32 s[8], int out_words, u32 o[8]) {
    auto f = [&](u32 x, u32 m) { return x & m; };
    switch (out_words) {
        case 4: {
            auto mix = [&](u32 a0, u32 a1, u32 a2, u32 a3, int n) {
                return rotl(f(a0, 0xFFu) | f(a1, 0xFF00u) | f(a2, 0xFF0000u) | f(a3, 0xFF000000u), n);
            };
            o[0] = s[0] + mix(s[7], s[4], s[5], s[6], 24);
            o[1] = s[1] + mix(s[6], s[7], s[4], s[5], 16);
            o[2] = s[2] + mix(s[5], s[6], s[7], s[4], 8);
            o[3] = s[3] + mix(s[4], s[5], s[6], s[7], 0);
            break;
        }
        case 5: {
            // 6/7-bit fields of s5, s6, s7 at bit offsets 0, 6, 12, 19, 25
            const u32 m[5] = {0x0000003Fu, 0x00000FC0u, 0x0007F000u, 0x01F80000u, 0xFE000000u};
            auto mix = [&](int i) {
                const u32 t = f(s[5], m[(i + 3) % 5]) | f(s[6], m[(i + 4) % 5]) | f(s[7], m[i]);
                switch (i) {
                    case 0: return rotl(t, 13);
                    case 1: return rotl(t, 7);
                    case 2: return t;
                    case 3: return t >> 6;
                    default: return t >> 12;
                }
            };
            for (int i = 0; i < 5; ++i) o[i] = s[i] + mix(i);
            break;
        }
        case 6: {
            o[0] = s[0] + rotl(f(s[6], 0xFC000000u) | f(s[7], 0x1Fu), 6);
            o[1] = s[1] + (f(s[6], 0x1Fu) | f(s[7], 0x3E0u));
            o[2] = s[2] + ((f(s[6], 0x3E0u) | f(s[7], 0xFC00u)) >> 5);
            o[3] = s[3] + ((f(s[6], 0xFC00u) | f(s[7], 0x1F0000u)) >> 10);
            o[4] = s[4] + ((f(s[6], 0x1F0000u) | f(s[7], 0x3E00000u)) >> 16);
            o[5] = s[5] + ((f(s[6], 0x3E00000u) | f(s[7], 0xFC000000u)) >> 21);
            break;
        }
        case 7: {
            const int sh[7] = {27, 22, 18, 13, 9, 4, 0};
            const u32 mk[7] = {0x1F, 0x1F, 0x0F, 0x1F, 0x0F, 0x1F, 0x0F};
            for (int i = 0; i < 7; ++i) o[i] = s[i] + ((s[7] >> sh[i]) & mk[i]);
            break;
        }
        default:
            for (int i = 0; i < 8; ++i) o[i] = s[i];
    }
}

// ------------------------------------------------------------------ Lyra2 sponge

constexpr int kBlockWords = 12;  // 768-bit rate
constexpr int kSafeWords = 8;    // 512-bit blocks while absorbing the input (keeps the IV half intact)

inline u64 rotr64(u64 x, int n) { return (x >> n) | (x << (64 - n)); }

struct Sponge {
    u64 v[16];
    Sponge() {
        // BLAKE2b IV (= SHA-512 IV) in the capacity half
        static const u64 iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                  0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                  0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
        std::memset(v, 0, 64);
        std::memcpy(v + 8, iv, 64);
    }
    static void g(u64& a, u64& b, u64& c, u64& d) {
        a += b; d = rotr64(d ^ a, 32);
        c += d; b = rotr64(b ^ c, 24);
        a += b; d = rotr64(d ^ a, 16);
        c += d; b = rotr64(b ^ c, 63);
    }
    // BLAKE2b rounds without message words or counters
    void rounds(int n) {
        for (int r = 0; r < n; ++r) {
            g(v[0], v[4], v[8], v[12]);
            g(v[1], v[5], v[9], v[13]);
            g(v[2], v[6], v[10], v[14]);
            g(v[3], v[7], v[11], v[15]);
            g(v[0], v[5], v[10], v[15]);
            g(v[1], v[6], v[11], v[12]);
            g(v[2], v[7], v[8], v[13]);
            g(v[3], v[4], v[9], v[14]);
        }
    }
    void absorb(const u64* in, int words) {
        for (int i = 0; i < words; ++i) v[i] ^= in[i];
        rounds(12);
    }
    void squeeze(u8* out, u64 len) {
        while (len >= u64(kBlockWords * 8)) {
            std::memcpy(out, v, kBlockWords * 8);
            rounds(12);
            out += kBlockWords * 8;
            len -= kBlockWords * 8;
        }
        std::memcpy(out, v, size_t(len));
    }
};

}  // namespace

std::vector<u8> haval_hash(const u8* data, size_t n, int passes, int out_bits) {
    if (passes < 3 || passes > 5 || out_bits < 128 || out_bits > 256 || out_bits % 32)
        throw std::invalid_argument("HAVAL: passes 3..5, output 128/160/192/224/256 bits");
    const int out_words = out_bits / 32;
    u32 s[8];
    std::memcpy(s, pi_words().w, sizeof s);
    size_t off = 0;
    for (; off + 128 <= n; off += 128) haval_block(s, data + off, passes);
    // tail: 0x01 pad byte, zeros up to byte 118, then VERSION=1|PASS<<3, FPTLEN<<6 as
    // (out_words<<3), and the 64-bit message bit length
    u8 buf[256] = {0};
    const size_t rem = n - off;
    std::memcpy(buf, data + off, rem);
    buf[rem] = 0x01;
    const size_t total = rem + 1 > 118 ? 256 : 128;
    buf[total - 10] = u8(0x01 | (passes << 3));
    buf[total - 9] = u8(out_words << 3);
    const u64 bits = u64(n) << 3;
    for (int i = 0; i < 8; ++i) buf[total - 8 + size_t(i)] = u8(bits >> (8 * i));
    for (size_t b = 0; b < total; b += 128) haval_block(s, buf + b, passes);
    u32 o[8];
    haval_fold(s, out_words, o);
    std::vector<u8> out(size_t(out_words) * 4);
    for (int i = 0; i < out_words; ++i) store_le32(out.data() + 4 * i, o[i]);
    return out;
}

std::vector<u8> lyra2_hash(const u8* pwd, size_t pwdlen, const u8* salt, size_t saltlen, u64 klen, u64 time_cost,
                           u64 n_rows, u64 n_cols, bool old_absorb) {
    if (n_rows < 4 || (n_rows & (n_rows - 1)) || n_cols < 1 || n_rows * n_cols > (u64(1) << 24)) return {};
    const u64 row_words = u64(kBlockWords) * n_cols;
    std::vector<u64> m(size_t(n_rows * row_words), 0);
    auto row = [&](u64 r) { return m.data() + r * row_words; };

    // pad10*1(pwd || salt || kLen, pwdlen, saltlen, timeCost, nRows, nCols) in 64-byte blocks, staged in
    // the matrix's first row(s) as the reference does (the setup phase overwrites it)
    const u64 n_blocks = (saltlen + pwdlen + 6 * 8) / (kSafeWords * 8) + 1;
    const u64 last_block = old_absorb ? (n_blocks - 1) * 64 : (n_blocks - 1) * kSafeWords;
    if ((last_block + kSafeWords) * 8 > m.size() * 8 || n_blocks * kSafeWords * 8 > m.size() * 8) return {};
    {
        u8* p = reinterpret_cast<u8*>(m.data());
        std::memcpy(p, pwd, pwdlen);
        std::memcpy(p + pwdlen, salt, saltlen);
        const u64 params[6] = {klen, u64(pwdlen), u64(saltlen), time_cost, n_rows, n_cols};
        std::memcpy(p + pwdlen + saltlen, params, sizeof params);  // little-endian host words
        p[pwdlen + saltlen + sizeof params] = 0x80;                  // 10*1 padding
        p[n_blocks * kSafeWords * 8 - 1] ^= 0x01;
    }
    Sponge sp;
    for (u64 i = 0; i < n_blocks; ++i) sp.absorb(m.data() + i * (old_absorb ? 64 : kSafeWords), kSafeWords);

    // row 0: squeezed column blocks written last-to-first, one reduced round each
    for (u64 c = 0; c < n_cols; ++c) {
        std::memcpy(row(0) + (n_cols - 1 - c) * kBlockWords, sp.v, kBlockWords * 8);
        sp.rounds(1);
    }
    // row 1 = row 0 duplexed, written in reverse column order
    for (u64 c = 0; c < n_cols; ++c) {
        const u64* in = row(0) + c * kBlockWords;
        u64* out = row(1) + (n_cols - 1 - c) * kBlockWords;
        for (int k = 0; k < kBlockWords; ++k) sp.v[k] ^= in[k];
        sp.rounds(1);
        for (int k = 0; k < kBlockWords; ++k) out[k] = in[k] ^ sp.v[k];
    }
    // setup phase: row r from prev and a revisited row*, which is fed back rotated by one word
    auto duplex = [&](u64 prev, u64 star, u64 r, bool setup) {
        for (u64 c = 0; c < n_cols; ++c) {
            const u64* in = row(prev) + c * kBlockWords;
            u64* io = row(star) + c * kBlockWords;
            u64* out = row(r) + (setup ? (n_cols - 1 - c) : c) * kBlockWords;
            for (int k = 0; k < kBlockWords; ++k) sp.v[k] ^= in[k] + io[k];
            sp.rounds(1);
            for (int k = 0; k < kBlockWords; ++k) out[k] = setup ? in[k] ^ sp.v[k] : out[k] ^ sp.v[k];
            for (int k = 0; k < kBlockWords; ++k) io[k] ^= sp.v[(k + kBlockWords - 1) % kBlockWords];
        }
    };
    u64 prev = 1, star = 0, step = 1, window = 2;
    int64_t gap = 1;
    for (u64 r = 2; r < n_rows; ++r) {
        duplex(prev, star, r, true);
        star = (star + step) & (window - 1);
        prev = r;
        if (star == 0) {
            step = u64(int64_t(window) + gap);
            window *= 2;
            gap = -gap;
        }
    }
    // wandering phase: row* picked by the sponge state
    u64 r = 0;
    for (u64 tau = 1; tau <= time_cost; ++tau) {
        const u64 st = (tau % 2 == 0) ? u64(-1) : n_rows / 2 - 1;  // the reference's (row + step) % nRows in u64
        do {
            star = sp.v[0] % n_rows;
            duplex(prev, star, r, false);
            prev = r;
            r = (r + st) % n_rows;
        } while (r != 0);
    }
    sp.absorb(row(star), kBlockWords);
    std::vector<u8> out(static_cast<size_t>(klen));
    sp.squeeze(out.data(), klen);
    return out;
}

// ------------------------------------------------------------------ GOST R 34.11-2012 (Streebog)
// The reference's sph_gost256 / sph_gost512 (src/algo/gost_streebog.c; linked, never called from
// consensus). Its byte convention: the state, the message blocks and the digest are big-endian
// byte strings (byte 0 most significant), i.e. the standard's test vectors byte-reversed
// (tests/test_legacy_algos.py checks example M1 both ways). The LPS layer is one table lookup per
// state byte; the 8 x 256 table is expanded at first use from its GF(2) structure: 8 bases of the
// linear layer's images and one S-box code shared by all byte positions (tools/gost_compact_tables.py
// derives them from the reference's table).
namespace {

// basis[i][b]: LPS image of basis byte b at input byte position i
static const u64 kGostBasis[8][8] = {
    {0xe6f87e5c5b711fd0ULL, 0x258377800924fa16ULL, 0xc849e07e852ea4a8ULL, 0x5b4686a18f06c16aULL, 0xabda37a467815c66ULL, 0xf61796a81a686676ULL, 0xf5dc0b706391954bULL, 0xff5c629a68bd85c5ULL},
    {0xc811a8058c3f55deULL, 0x65f5b43196b50619ULL, 0xf74f96b1d6706e43ULL, 0x859d1e8bcb43d336ULL, 0xf9c7bf99c295fcfdULL, 0xa21fd5a1de4b630fULL, 0xcdb3ef763b8b456dULL, 0xb27c73be5f31913cULL},
    {0x45b268a93acde4ccULL, 0xaf7f0be884549d08ULL, 0x048354b3c1468263ULL, 0x925435c2c80efed2ULL, 0x167a33920c60f14dULL, 0xfb123b52ea03e584ULL, 0x4a0cab53fdbb9007ULL, 0xcb48ec558f0cb32aULL},
    {0x05ba7bc82c9b3220ULL, 0x31a54665f8b65e4fULL, 0xb1b651f77547f4d4ULL, 0x8bfa0d857ba46682ULL, 0x990faef908eb79c9ULL, 0xa15e37a247f4a62dULL, 0x76857dcd5d27741eULL, 0xbe65dcb201f7a2b4ULL},
    {0x3ef29d249b2c0a19ULL, 0xe9e16322b6f8622fULL, 0x5536994047757f7aULL, 0x9f4d56d5a47b0b33ULL, 0xb8f5057deb082fb2ULL, 0xcc48c10bf4475f53ULL, 0x373088d4275dec3aULL, 0x173d232cf7016151ULL},
    {0x8ab0a96846e06a6dULL, 0x43c7e80b4bf0b33aULL, 0x08c9b3546b161ee5ULL, 0x39f1c235eba990beULL, 0x2c209233614569aaULL, 0xeb01523b6fc3289aULL, 0x946953ab935aceddULL, 0x8b0455eca12ba052ULL},
    {0x7e37e62dfc7d40c3ULL, 0x776f25a4ee939e5bULL, 0xe045c850dd8fb5adULL, 0x86ed5ba711ff1952ULL, 0x37e0ab256e408ffbULL, 0x9607f6c031025a7aULL, 0x0b02f5e116d23c9dULL, 0x621cff27c40875f5ULL},
    {0xd031c397ce553fe6ULL, 0x16ba5b01b006b525ULL, 0xa89bade6296e70c8ULL, 0x6a1f525d77d3435bULL, 0x660efb2a17fc95abULL, 0x76327a9e97634bf6ULL, 0x4bad9d6462458bf5ULL, 0xc5c8f542669131ffULL},
};
// code[x]: the S-box output of x in that basis
static const u8 kGostCode[256] = {
      1,   2,   4,   8,   7,  16,  32,  64,  73, 128, 100,  76,  35, 173,  67,  51,
     74, 148, 206,  97,  60, 193, 150, 181, 109, 104, 227, 152, 102,  33,  48, 238,
    111, 169, 151,  94, 205,  59,  47,   5,  63, 234, 194, 247, 149,  45, 251,  21,
    110,  81,  38, 211, 224,  83, 214,  58, 101, 135,   9, 187,  24, 165, 237, 225,
    108,  78, 231, 217,  65,  79,  93, 189, 232, 130, 117,  28,  44, 167,  42,  12,
    113, 220, 233, 145, 140, 207, 185,   3, 219, 250,  46, 153, 248,  87,  22,  90,
     75,  23,  82, 137,  37,  91, 157, 139, 197,  26,  80,  61, 213, 222,  57,  50,
     43, 178, 132, 239,  10,  99, 184,  53,  27, 183, 166,  18, 200, 253, 226, 188,
     34, 160, 107, 155, 228, 182, 218,  98, 174, 125, 131, 171,  19,  14, 190,  11,
    235, 196,  36,  15, 118, 116,  31, 208,  41, 103, 164, 244,  56,   6, 170, 123,
    114, 127, 249, 215, 204,   0, 223, 146, 143, 147, 129,  52, 186, 243,  77, 252,
    216, 191, 180,  17,  96,  29, 154, 236, 221,  49,  84,  62,  88, 136,  89, 138,
     72, 120,  20, 209, 119, 245, 199, 134,  13,  69, 126, 168, 158,  71, 163, 179,
    198, 162,  25, 112,  30, 201,  66,  39, 240, 255, 144,  55, 105, 106, 124, 212,
     40, 241, 177, 121, 202, 175, 161, 115,  68, 176,  70, 230, 246, 133,  54, 210,
     85,  95, 159, 192, 142, 141,  92, 195, 203, 156, 254, 229, 172,  86, 242, 122,
};
// iteration constants C_1..C_12 as little-endian words of the state layout
static const u64 kGostC[12][8] = {
    {0xe9daca1eda5b08b1ULL, 0x1f7c65c0812fcbebULL, 0x16d0452e43766a2fULL, 0xfcc485758db84e71ULL, 0x0169679291e07c4bULL, 0x15d360a4082a42a2ULL, 0x234d74cc36747605ULL, 0x0745a6f2596580ddULL},
    {0x1a2f9da98ab5a36fULL, 0xd7b5700f469de34fULL, 0x982b230a72eafef3ULL, 0x3101b5160f5ed561ULL, 0x5899d6126b17b59aULL, 0xcaa70adbc261b55cULL, 0x56cdcbd71ba2dd55ULL, 0xb79bb121700479e6ULL},
    {0xc72fce2bacdc74f5ULL, 0x35843d6a28fc390aULL, 0x8b1f9c525f5ef106ULL, 0x7b7b29b11475eaf2ULL, 0xb19e3590e40fe2d3ULL, 0x09db6260373ac9c1ULL, 0x31db7a8643f4b6c2ULL, 0xb20aba0af5961e99ULL},
    {0xd26615e8b3df1fefULL, 0xdde4715da0e148f9ULL, 0x7d3c5c337e858e48ULL, 0x3f355e68ad1c729dULL, 0x75d603ed822cd7a9ULL, 0xbe0352933313b7d8ULL, 0xf137e893a1ea5334ULL, 0x2ed1e384bcbe0c22ULL},
    {0x994747adac6bea4bULL, 0x6323a96c0c413f9aULL, 0x4a1086161f1c157fULL, 0xbdff0f80d7359e35ULL, 0xa3f53a254717cdbfULL, 0x161a2723b700ffdfULL, 0xf563eaa97ea2567aULL, 0x57fe6c7cfd581760ULL},
    {0xd9d33a1daeae4faeULL, 0xc039307a3bc3a46fULL, 0x6ca44251f9c4662dULL, 0xc68ef09ab49a7f18ULL, 0xb4b79a1cb7a6facfULL, 0xb6c6bec2661ff20aULL, 0x354f903672c571bfULL, 0x6e7d64467a4068faULL},
    {0xecc5aaee160ec7f4ULL, 0x540924bffe86ac51ULL, 0xc987bfe6c7c69e39ULL, 0xc9937a19333e47d3ULL, 0x372c822dc5ab9209ULL, 0x04054a2883694706ULL, 0xf34a3ca24c451735ULL, 0x93d4143a4d568688ULL},
    {0xa7c9934d425b1f9bULL, 0x41416e0c02aae703ULL, 0x1ede369c71f8b74eULL, 0x9ac4db4d3b44b489ULL, 0x90069b92cb2b89f4ULL, 0x2fc4a5d12b8dd169ULL, 0xd9a8515935c2ac36ULL, 0x1ee702bfd40d7fa4ULL},
    {0x9b223116545a8f37ULL, 0xde5f16ecd89a4c94ULL, 0x244289251b3a7d3aULL, 0x84090de0b755d93cULL, 0xb1ceb2db0b440a80ULL, 0x549c07a69a8a2b7bULL, 0x602a1fcb92dc380eULL, 0xdb5a238351446172ULL},
    {0x526f0580a6debeabULL, 0xf3f3e4b248e52a38ULL, 0xdb788aff1ce74189ULL, 0x0361331b8ae1ff1fULL, 0x4b3369af0267e79fULL, 0xf452763b306c1e7aULL, 0xc3b63b15d1fa9836ULL, 0xed9c4598fbc7b474ULL},
    {0xfb89c8efd09ecd7bULL, 0x94fe5a63cdc60230ULL, 0x6107abebbb6bfad8ULL, 0x7966841421800120ULL, 0xcab948eaef711d8aULL, 0x986e477d1dcdbaefULL, 0x5dd86fc04a59a2deULL, 0x1b2df381cda4ca6bULL},
    {0xba3116f167e78e37ULL, 0x7ab14904b08013d2ULL, 0x771ddfbc323ca4cdULL, 0x9b9f2130d41220f8ULL, 0x86cc91189def805dULL, 0x5228e188aaa41de7ULL, 0x991bb2d9d517f4faULL, 0x20d71bf14a92bc48ULL},
};

struct GostLps {
    u64 t[8][256];
    GostLps() {
        for (int i = 0; i < 8; ++i)
            for (int x = 0; x < 256; ++x) {
                u64 acc = 0;
                for (int b = 0; b < 8; ++b)
                    if (kGostCode[x] >> b & 1) acc ^= kGostBasis[i][b];
                t[i][x] = acc;
            }
    }
};

const GostLps& gost_lps() {
    static const GostLps tab;
    return tab;
}

// The 512-bit state as 8 little-endian words: byte j of the byte string is byte j % 8 of w[j / 8].
struct G512 {
    u64 w[8];
};

inline G512 gost_xor(const G512& a, const G512& b) {
    G512 r;
    for (int k = 0; k < 8; ++k) r.w[k] = a.w[k] ^ b.w[k];
    return r;
}

// S, P and L in one pass: output word k takes byte k of every input word, position 7 - word.
inline G512 gost_lps_apply(const G512& s) {
    const GostLps& T = gost_lps();
    G512 r;
    for (int k = 0; k < 8; ++k) {
        u64 acc = 0;
        for (int i = 0; i < 8; ++i) acc ^= T.t[i][(s.w[7 - i] >> (8 * k)) & 0xFF];
        r.w[k] = acc;
    }
    return r;
}

inline G512 gost_from_bytes(const u8* b) {
    G512 r;
    std::memcpy(r.w, b, 64);  // little-endian host: byte j -> byte j % 8 of word j / 8
    return r;
}

// a + b mod 2^512 on the big-endian byte strings
inline G512 gost_add(const G512& a, const G512& b) {
    u8 x[64], y[64], z[64];
    std::memcpy(x, a.w, 64);
    std::memcpy(y, b.w, 64);
    unsigned carry = 0;
    for (int j = 63; j >= 0; --j) {
        const unsigned t = unsigned(x[j]) + y[j] + carry;
        z[j] = u8(t);
        carry = t >> 8;
    }
    return gost_from_bytes(z);
}

// g_N(h, m): E over the key N ^ h, then the Miyaguchi-Preneel feed-forward
G512 gost_g(const G512& n, const G512& h, const G512& m) {
    G512 k = gost_lps_apply(gost_xor(n, h));
    G512 s = gost_xor(m, k);
    for (int i = 0; i < 12; ++i) {
        s = gost_lps_apply(s);
        G512 c;
        std::memcpy(c.w, kGostC[i], 64);
        k = gost_lps_apply(gost_xor(k, c));
        s = gost_xor(s, k);
    }
    return gost_xor(gost_xor(s, h), m);
}

}  // namespace

std::vector<u8> gost_streebog(const u8* data, size_t n, int out_bits) {
    if (out_bits != 256 && out_bits != 512) throw std::invalid_argument("gost: out_bits is 256 or 512");
    G512 h;
    for (u64& x : h.w) x = out_bits == 256 ? 0x0101010101010101ULL : 0;
    G512 nsum{}, sigma{}, zero{};
    G512 step{};  // 512 as a big-endian byte string: byte 62 = 0x02
    reinterpret_cast<u8*>(step.w)[62] = 0x02;
    // full 64-byte blocks from the END of the message (the big-endian number's low end)
    size_t rem = n;
    while (rem >= 64) {
        const G512 m = gost_from_bytes(data + rem - 64);
        h = gost_g(nsum, h, m);
        nsum = gost_add(nsum, step);
        sigma = gost_add(sigma, m);
        rem -= 64;
    }
    // the remaining head, right-aligned, with a 1 bit just above it
    u8 last[64] = {0};
    std::memcpy(last + 64 - rem, data, rem);
    last[63 - rem] |= 1;
    const G512 m = gost_from_bytes(last);
    h = gost_g(nsum, h, m);
    G512 bits{};
    const size_t nb = rem * 8;
    reinterpret_cast<u8*>(bits.w)[63] = u8(nb);
    reinterpret_cast<u8*>(bits.w)[62] = u8(nb >> 8);
    nsum = gost_add(nsum, bits);
    sigma = gost_add(sigma, m);
    h = gost_g(zero, h, nsum);
    h = gost_g(zero, h, sigma);
    std::vector<u8> out(size_t(out_bits / 8));
    std::memcpy(out.data(), h.w, out.size());  // the first bytes of the big-endian string
    return out;
}

}  // namespace nodexa
