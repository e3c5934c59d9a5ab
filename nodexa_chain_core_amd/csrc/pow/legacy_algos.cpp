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

}  // namespace nodexa
