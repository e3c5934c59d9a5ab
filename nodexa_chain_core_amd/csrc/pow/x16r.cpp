#include "x16r.hpp"
#include "x16r_prims.hpp"

#include <atomic>
#include <stdexcept>
#include <thread>
#include <utility>
#include <vector>

namespace nodexa {

// ------------------------------------------------------------------ BLAKE-512
// SHA-3 finalist BLAKE (Aumasson, Henzen, Meier, Phan), 16 rounds, 64-bit words.
namespace {
const u64 kBlakeIV[8] = {0x6A09E667F3BCC908ULL, 0xBB67AE8584CAA73BULL, 0x3C6EF372FE94F82BULL, 0xA54FF53A5F1D36F1ULL,
                         0x510E527FADE682D1ULL, 0x9B05688C2B3E6C1FULL, 0x1F83D9ABFB41BD6BULL, 0x5BE0CD19137E2179ULL};
const u64 kBlakeC[16] = {0x243F6A8885A308D3ULL, 0x13198A2E03707344ULL, 0xA4093822299F31D0ULL, 0x082EFA98EC4E6C89ULL,
                         0x452821E638D01377ULL, 0xBE5466CF34E90C6CULL, 0xC0AC29B7C97C50DDULL, 0x3F84D5B5B5470917ULL,
                         0x9216D5D98979FB1BULL, 0xD1310BA698DFB5ACULL, 0x2FFD72DBD01ADFB7ULL, 0xB8E1AFED6A267E96ULL,
                         0xBA7C9045F12C7F99ULL, 0x24A19947B3916CF7ULL, 0x0801F2E2858EFC16ULL, 0x636920D871574E69ULL};
const u8 kSigma[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

inline u64 rotr64(u64 x, int n) { return (x >> n) | (x << (64 - n)); }

void blake512_compress(u64 h[8], const u8* block, u64 t0, u64 t1) {
    u64 m[16], v[16];
    for (int i = 0; i < 16; ++i) m[i] = load_be64(block + 8 * i);
    for (int i = 0; i < 8; ++i) v[i] = h[i];
    v[8] = kBlakeC[0]; v[9] = kBlakeC[1]; v[10] = kBlakeC[2]; v[11] = kBlakeC[3];
    v[12] = t0 ^ kBlakeC[4]; v[13] = t0 ^ kBlakeC[5]; v[14] = t1 ^ kBlakeC[6]; v[15] = t1 ^ kBlakeC[7];
    auto G = [&](int r, int i, int a, int b, int c, int d) {
        const u8* s = kSigma[r % 10];
        v[a] = v[a] + v[b] + (m[s[2 * i]] ^ kBlakeC[s[2 * i + 1]]);
        v[d] = rotr64(v[d] ^ v[a], 32);
        v[c] = v[c] + v[d];
        v[b] = rotr64(v[b] ^ v[c], 25);
        v[a] = v[a] + v[b] + (m[s[2 * i + 1]] ^ kBlakeC[s[2 * i]]);
        v[d] = rotr64(v[d] ^ v[a], 16);
        v[c] = v[c] + v[d];
        v[b] = rotr64(v[b] ^ v[c], 11);
    };
    for (int r = 0; r < 16; ++r) {
        G(r, 0, 0, 4, 8, 12); G(r, 1, 1, 5, 9, 13); G(r, 2, 2, 6, 10, 14); G(r, 3, 3, 7, 11, 15);
        G(r, 4, 0, 5, 10, 15); G(r, 5, 1, 6, 11, 12); G(r, 6, 2, 7, 8, 13); G(r, 7, 3, 4, 9, 14);
    }
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}
}  // namespace

Hash512 blake512(const u8* data, size_t n) {
    u64 h[8];
    for (int i = 0; i < 8; ++i) h[i] = kBlakeIV[i];
    const u64 total_bits = u64(n) * 8;
    u64 t = 0;
    while (n >= 128) {
        t += 1024;
        blake512_compress(h, data, t, 0);
        data += 128;
        n -= 128;
    }
    u8 buf[256] = {0};
    std::memcpy(buf, data, n);
    buf[n] = 0x80;
    const bool two = n >= 112;  // 111 payload bytes + 1 flag + 16 length
    const size_t len = two ? 256 : 128;
    buf[len - 17] |= 0x01;
    store_be64(buf + len - 8, total_bits);
    // length high 64 bits (buf + len - 16) stay zero
    if (!two) {
        blake512_compress(h, buf, n ? total_bits : 0, 0);
    } else {
        blake512_compress(h, buf, total_bits, 0);
        blake512_compress(h, buf + 128, 0, 0);
    }
    Hash512 out;
    for (int i = 0; i < 8; ++i) store_be64(out.bytes + 8 * i, h[i]);
    return out;
}

// ------------------------------------------------------------------ SHA-512 (FIPS 180-4)
namespace {
constexpr u64 kSha512K[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, 0x3956c25bf348b538ULL,
    0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, 0xd807aa98a3030242ULL, 0x12835b0145706fbeULL,
    0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, 0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL,
    0xc19bf174cf692694ULL, 0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, 0x983e5152ee66dfabULL,
    0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, 0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL,
    0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, 0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL,
    0x53380d139d95b3dfULL, 0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, 0xd192e819d6ef5218ULL,
    0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, 0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL,
    0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, 0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL,
    0x682e6ff3d6b2b8a3ULL, 0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, 0xca273eceea26619cULL,
    0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, 0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL,
    0x113f9804bef90daeULL, 0x1b710b35131c471bULL, 0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL,
    0x431d67c49c100d4cULL, 0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

// Rounds unrolled at compile time over a rolling 16-word schedule.
template <int I>
inline void sha512_round(u64 (&v)[8], u64 (&w)[16]) {
    if constexpr (I >= 16) {
        const u64 a = w[(I - 15) & 15], b = w[(I - 2) & 15];
        w[I & 15] += (rotr64(a, 1) ^ rotr64(a, 8) ^ (a >> 7)) + w[(I - 7) & 15] +
                     (rotr64(b, 19) ^ rotr64(b, 61) ^ (b >> 6));
    }
    u64 &A = v[(80 - I) & 7], &B = v[(81 - I) & 7], &C = v[(82 - I) & 7], &D = v[(83 - I) & 7];
    u64 &E = v[(84 - I) & 7], &F = v[(85 - I) & 7], &G = v[(86 - I) & 7], &H = v[(87 - I) & 7];
    const u64 t1 = H + (rotr64(E, 14) ^ rotr64(E, 18) ^ rotr64(E, 41)) + ((E & F) ^ (~E & G)) + kSha512K[I] + w[I & 15];
    const u64 t2 = (rotr64(A, 28) ^ rotr64(A, 34) ^ rotr64(A, 39)) + ((A & B) ^ (A & C) ^ (B & C));
    D += t1;
    H = t1 + t2;
}

template <int... I>
inline void sha512_rounds(std::integer_sequence<int, I...>, u64 (&v)[8], u64 (&w)[16]) {
    (sha512_round<I>(v, w), ...);
}

void sha512_compress(u64 s[8], const u8* block) {
    u64 w[16], v[8];
    for (int i = 0; i < 16; ++i) w[i] = load_be64(block + 8 * i);
    for (int i = 0; i < 8; ++i) v[i] = s[i];
    sha512_rounds(std::make_integer_sequence<int, 80>{}, v, w);
    for (int i = 0; i < 8; ++i) s[i] += v[i];
}
}  // namespace

Hash512 sha512_hash(const u8* data, size_t n) {
    u64 s[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    const u64 total = u64(n);
    while (n >= 128) {
        sha512_compress(s, data);
        data += 128;
        n -= 128;
    }
    u8 buf[256] = {0};
    std::memcpy(buf, data, n);
    buf[n] = 0x80;
    const size_t len = (n < 112) ? 128 : 256;
    store_be64(buf + len - 8, total * 8);
    sha512_compress(s, buf);
    if (len == 256) sha512_compress(s, buf + 128);
    Hash512 out;
    for (int i = 0; i < 8; ++i) store_be64(out.bytes + 8 * i, s[i]);
    return out;
}

// ------------------------------------------------------------------ dispatcher
int x16r_selection(const u8 prev_le[32], int index) {
    // GetNibble(48 + index): nibble 63-(48+index) of the little-endian storage
    const int i = 63 - (48 + index);
    return (i % 2 == 1) ? (prev_le[i / 2] >> 4) : (prev_le[i / 2] & 0x0F);
}

bool x16r_slot_available(int algo) { return algo >= 0 && algo <= 16; }

Hash512 x16r_single(int algo, const u8* data, size_t n) {
    switch (algo) {
        case 0: return blake512(data, n);
        case 1: return bmw512(data, n);
        case 2: return groestl512(data, n);
        case 3: return jh512(data, n);
        case 4: return keccak512(data, n);
        case 5: return skein512(data, n);
        case 6: return luffa512(data, n);
        case 7: return cubehash512(data, n);
        case 8: return shavite512(data, n);
        case 9: return simd512(data, n);
        case 10: return echo512(data, n);
        case 11: return hamsi512(data, n);
        case 12: return fugue512(data, n);
        case 13: return shabal512(data, n);
        case 14: return whirlpool512(data, n);
        case 15: return sha512_hash(data, n);
        case 16: return tiger192_padded(data, n);
        default: throw std::invalid_argument("X16R slot out of range: " + std::to_string(algo));
    }
}

void x16r_hash(const u8* data, size_t n, const u8 prev_le[32], bool v2, u8 out[32]) {
    Hash512 h;
    static const u8 kEmpty[1] = {0};
    const u8* in = n ? data : kEmpty;  // an empty message may come with a null pointer
    size_t len = n;
    for (int i = 0; i < 16; ++i) {
        const int sel = x16r_selection(prev_le, i);
        if (v2 && (sel == 4 || sel == 6 || sel == 15)) {
            const Hash512 t = x16r_single(16, in, len);
            h = x16r_single(sel, t.bytes, 64);
        } else {
            h = x16r_single(sel, in, len);
        }
        in = h.bytes;
        len = 64;
    }
    std::memcpy(out, h.bytes, 32);
}

X16rSearchResult x16r_search(const u8 header80[80], bool v2, const u8 target_le[32], u32 start, u64 count,
                             int threads) {
    // generateBlocks' legacy loop (src/rpc/mining.cpp:141-149: ++nNonce until
    // CheckProofOfWork) split over host threads in interleaved nonce order; the
    // lowest qualifying nonce of the window wins, so the result is deterministic.
    if (threads <= 0) threads = int(std::max(1u, std::thread::hardware_concurrency()));
    const u8* prev = header80 + 4;
    std::atomic<u64> best{~u64(0)};
    std::atomic<u64> done{0};
    auto le_cmp = [](const u8* a, const u8* b) {  // a <= b as little-endian 256-bit
        for (int i = 31; i >= 0; --i)
            if (a[i] != b[i]) return a[i] < b[i];
        return true;
    };
    auto worker = [&](int t) {
        u8 hdr[80];
        std::memcpy(hdr, header80, 80);
        u64 local = 0;
        for (u64 k = u64(t); k < count; k += u64(threads)) {
            if (k > best.load(std::memory_order_relaxed)) break;
            store_le32(hdr + 76, u32(start + k));
            u8 out[32];
            x16r_hash(hdr, 80, prev, v2, out);
            ++local;
            if (le_cmp(out, target_le)) {
                u64 cur = best.load();
                while (k < cur && !best.compare_exchange_weak(cur, k)) {
                }
                break;
            }
        }
        done += local;
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) pool.emplace_back(worker, t);
    for (auto& th : pool) th.join();
    X16rSearchResult r;
    r.hashes = done.load();
    if (best.load() != ~u64(0)) {
        r.found = true;
        r.nonce = u32(start + best.load());
        u8 hdr[80];
        std::memcpy(hdr, header80, 80);
        store_le32(hdr + 76, r.nonce);
        x16r_hash(hdr, 80, prev, v2, r.hash);
    }
    return r;
}

}  // namespace nodexa
