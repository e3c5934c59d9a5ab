// X16R add-rotate-xor primitives: CubeHash16/32-512, Skein-512-512, Shabal-512, BMW-512.
//
// Parity: sph_cubehash512 / sph_skein512 / sph_shabal512 / sph_bmw512 as linked by
// HashX16R (src/hash.h:335-462). Written from the SHA-3 round-2 specifications.
#include "x16r_prims.hpp"

namespace nodexa {

// ================================================================ CubeHash16/32-512
// 32 x u32 state; r = 16 rounds per 32-byte block; IV = 10r rounds over (h/8, b, r).
namespace {

void cubehash_rounds(u32 x[32], int rounds) {
    for (int r = 0; r < rounds; ++r) {
        for (int j = 0; j < 16; ++j) x[16 + j] += x[j];
        for (int j = 0; j < 16; ++j) x[j] = rotl32(x[j], 7);
        for (int j = 0; j < 8; ++j) std::swap(x[j], x[j + 8]);
        for (int j = 0; j < 16; ++j) x[j] ^= x[16 + j];
        for (int j = 16; j < 32; ++j)
            if (!(j & 2)) std::swap(x[j], x[j + 2]);
        for (int j = 0; j < 16; ++j) x[16 + j] += x[j];
        for (int j = 0; j < 16; ++j) x[j] = rotl32(x[j], 11);
        for (int j = 0; j < 16; ++j)
            if (!(j & 4)) std::swap(x[j], x[j + 4]);
        for (int j = 0; j < 16; ++j) x[j] ^= x[16 + j];
        for (int j = 16; j < 32; j += 2) std::swap(x[j], x[j + 1]);
    }
}

struct CubeIV {
    u32 x[32];
    CubeIV() {
        for (auto& w : x) w = 0;
        x[0] = 64; x[1] = 32; x[2] = 16;
        cubehash_rounds(x, 160);
    }
};

}  // namespace

Hash512 cubehash512(const u8* data, size_t n) {
    static const CubeIV iv;
    u32 x[32];
    std::memcpy(x, iv.x, sizeof x);
    auto block = [&](const u8* p) {
        for (int i = 0; i < 8; ++i) x[i] ^= load_le32(p + 4 * i);
        cubehash_rounds(x, 16);
    };
    for (; n >= 32; n -= 32, data += 32) block(data);
    u8 last[32] = {0};
    std::memcpy(last, data, n);
    last[n] = 0x80;
    block(last);
    x[31] ^= 1;
    cubehash_rounds(x, 160);
    Hash512 out;
    for (int i = 0; i < 16; ++i) store_le32(out.bytes + 4 * i, x[i]);
    return out;
}

// ================================================================ Skein-512-512 (v1.3)
// UBI chaining over Threefish-512 (72 rounds, key injection every 4 rounds).
namespace {

constexpr int kSkeinRot[8][4] = {{46, 36, 19, 37}, {33, 27, 14, 42}, {17, 49, 36, 39}, {44, 9, 54, 56},
                                 {39, 30, 34, 24}, {13, 50, 10, 17}, {25, 29, 39, 43}, {8, 35, 56, 22}};
constexpr int kSkeinPerm[8] = {2, 1, 4, 7, 6, 5, 0, 3};
constexpr u64 kSkeinTypeCfg = 4, kSkeinTypeMsg = 48, kSkeinTypeOut = 63;

void threefish512(const u64 key[8], const u64 tweak[2], const u64 in[8], u64 out[8]) {
    u64 k[9], t[3] = {tweak[0], tweak[1], tweak[0] ^ tweak[1]};
    k[8] = 0x1BD11BDAA9FC1A22ULL;
    for (int i = 0; i < 8; ++i) { k[i] = key[i]; k[8] ^= key[i]; }
    u64 v[8];
    auto inject = [&](int s) {
        for (int i = 0; i < 8; ++i) v[i] += k[(s + i) % 9];
        v[5] += t[s % 3];
        v[6] += t[(s + 1) % 3];
        v[7] += u64(s);
    };
    for (int i = 0; i < 8; ++i) v[i] = in[i];
    inject(0);
    for (int d = 0; d < 72; ++d) {
        for (int j = 0; j < 4; ++j) {
            v[2 * j] += v[2 * j + 1];
            v[2 * j + 1] = rotl64(v[2 * j + 1], kSkeinRot[d % 8][j]) ^ v[2 * j];
        }
        u64 p[8];
        for (int i = 0; i < 8; ++i) p[i] = v[kSkeinPerm[i]];
        std::memcpy(v, p, sizeof v);
        if (d % 4 == 3) inject(d / 4 + 1);
    }
    for (int i = 0; i < 8; ++i) out[i] = v[i];
}

// UBI(G, M, type): chain over 64-byte blocks, G updated in place.
void skein_ubi(u64 g[8], const u8* m, size_t n, u64 type) {
    u64 pos = 0;
    bool first = true;
    do {
        const size_t take = n > 64 ? 64 : n;
        u8 blk[64] = {0};
        std::memcpy(blk, m, take);
        pos += take;
        m += take;
        n -= take;
        const bool final = n == 0;
        const u64 tw[2] = {pos, (type << 56) | (u64(first) << 62) | (u64(final) << 63)};
        u64 w[8], e[8];
        for (int i = 0; i < 8; ++i) w[i] = load_le64(blk + 8 * i);
        threefish512(g, tw, w, e);
        for (int i = 0; i < 8; ++i) g[i] = e[i] ^ w[i];
        first = false;
    } while (n > 0);
}

struct SkeinIV {
    u64 g[8] = {0};
    SkeinIV() {
        u8 cfg[32] = {'S', 'H', 'A', '3', 1, 0, 0, 0};
        store_le64(cfg + 8, 512);
        skein_ubi(g, cfg, 32, kSkeinTypeCfg);
    }
};

}  // namespace

Hash512 skein512(const u8* data, size_t n) {
    static const SkeinIV iv;
    u64 g[8];
    std::memcpy(g, iv.g, sizeof g);
    skein_ubi(g, data, n, kSkeinTypeMsg);
    u8 ctr[8] = {0};
    skein_ubi(g, ctr, 8, kSkeinTypeOut);
    Hash512 out;
    for (int i = 0; i < 8; ++i) store_le64(out.bytes + 8 * i, g[i]);
    return out;
}

// ================================================================ Shabal-512
// A[12], B[16], C[16], 64-bit block counter W; IV from two prefix blocks (W = -1, 0).
namespace {

struct Shabal {
    u32 A[12], B[16], C[16];
    u64 W;

    void perm(const u32 M[16]) {
        for (int i = 0; i < 16; ++i) B[i] = rotl32(B[i], 17);
        for (int j = 0; j < 3; ++j)
            for (int i = 0; i < 16; ++i) {
                const int a = (i + 16 * j) % 12, ap = (i + 16 * j + 11) % 12;
                u32 v = A[a] ^ (rotl32(A[ap], 15) * 5u) ^ C[(8 - i + 16) % 16];
                A[a] = (v * 3u) ^ B[(i + 13) % 16] ^ (B[(i + 9) % 16] & ~B[(i + 6) % 16]) ^ M[i];
                B[i] = ~(rotl32(B[i], 1) ^ A[a]);
            }
        for (int j = 0; j < 36; ++j) A[j % 12] += C[(j + 3) % 16];
    }
    void block(const u32 M[16], bool swap = true) {
        for (int i = 0; i < 16; ++i) B[i] += M[i];
        A[0] ^= u32(W);
        A[1] ^= u32(W >> 32);
        perm(M);
        for (int i = 0; i < 16; ++i) C[i] -= M[i];
        if (swap)
            for (int i = 0; i < 16; ++i) std::swap(B[i], C[i]);
    }
};

struct ShabalIV {
    Shabal s;
    ShabalIV() {
        std::memset(&s, 0, sizeof s);
        u32 M[16];
        s.W = ~u64(0);
        for (int i = 0; i < 16; ++i) M[i] = 512 + i;
        s.block(M);
        s.W = 0;
        for (int i = 0; i < 16; ++i) M[i] = 512 + 16 + i;
        s.block(M);
    }
};

}  // namespace

Hash512 shabal512(const u8* data, size_t n) {
    static const ShabalIV iv;
    Shabal s = iv.s;
    s.W = 1;
    u32 M[16];
    for (; n >= 64; n -= 64, data += 64) {
        for (int i = 0; i < 16; ++i) M[i] = load_le32(data + 4 * i);
        s.block(M);
        ++s.W;
    }
    u8 last[64] = {0};
    std::memcpy(last, data, n);
    last[n] = 0x80;
    for (int i = 0; i < 16; ++i) M[i] = load_le32(last + 4 * i);
    // final block, then three extra rounds of the same block with W frozen
    for (int i = 0; i < 16; ++i) s.B[i] += M[i];
    for (int k = 0; k < 4; ++k) {
        if (k) for (int i = 0; i < 16; ++i) std::swap(s.B[i], s.C[i]);
        s.A[0] ^= u32(s.W);
        s.A[1] ^= u32(s.W >> 32);
        s.perm(M);
    }
    Hash512 out;
    for (int i = 0; i < 16; ++i) store_le32(out.bytes + 4 * i, s.B[i]);
    return out;
}

// ================================================================ BMW-512 (Blue Midnight Wish)
// Double-pipe 16 x u64: f0 (bijective transform of M^H into Q[0..15]), f1 (two
// expansion functions for Q[16..31]), f2 (folding into the new pipe). Final step
// compresses the last pipe as a message under the constant pipe 0xaa..a0+j.
namespace {

// f0: W_i = sum of five (M^H)_j with signs; (index, sign) pairs, sign -1 = subtract.
struct WTerm { int idx[5]; int sgn[5]; };
const WTerm kBmwW[16] = {
    {{5, 7, 10, 13, 14}, {1, -1, 1, 1, 1}},  {{6, 8, 11, 14, 15}, {1, -1, 1, 1, -1}},
    {{0, 7, 9, 12, 15}, {1, 1, 1, -1, 1}},   {{0, 1, 8, 10, 13}, {1, -1, 1, -1, 1}},
    {{1, 2, 9, 11, 14}, {1, 1, 1, -1, -1}},  {{3, 2, 10, 12, 15}, {1, -1, 1, -1, 1}},
    {{4, 0, 3, 11, 13}, {1, -1, -1, -1, 1}}, {{1, 4, 5, 12, 14}, {1, -1, -1, -1, -1}},
    {{2, 5, 6, 13, 15}, {1, -1, -1, 1, -1}}, {{0, 3, 6, 7, 14}, {1, -1, 1, -1, 1}},
    {{8, 1, 4, 7, 15}, {1, -1, -1, -1, 1}},  {{8, 0, 2, 5, 9}, {1, -1, -1, -1, 1}},
    {{1, 3, 6, 9, 10}, {1, 1, -1, -1, 1}},   {{2, 4, 7, 10, 11}, {1, 1, 1, 1, 1}},
    {{3, 5, 8, 11, 12}, {1, -1, 1, -1, -1}}, {{12, 4, 6, 9, 13}, {1, -1, -1, -1, 1}}};

inline u64 bmw_s(int k, u64 x) {
    switch (k) {
        case 0: return (x >> 1) ^ (x << 3) ^ rotl64(x, 4) ^ rotl64(x, 37);
        case 1: return (x >> 1) ^ (x << 2) ^ rotl64(x, 13) ^ rotl64(x, 43);
        case 2: return (x >> 2) ^ (x << 1) ^ rotl64(x, 19) ^ rotl64(x, 53);
        case 3: return (x >> 2) ^ (x << 2) ^ rotl64(x, 28) ^ rotl64(x, 59);
        case 4: return (x >> 1) ^ x;
        default: return (x >> 2) ^ x;
    }
}

void bmw_compress(const u64 M[16], const u64 H[16], u64 out[16]) {
    u64 Q[32];
    for (int i = 0; i < 16; ++i) {
        u64 w = 0;
        for (int t = 0; t < 5; ++t) {
            const int j = kBmwW[i].idx[t];
            const u64 v = M[j] ^ H[j];
            w = (kBmwW[i].sgn[t] > 0) ? w + v : w - v;
        }
        Q[i] = bmw_s(i % 5, w) + H[(i + 1) & 15];
    }
    static const int kRot[7] = {5, 11, 27, 32, 37, 43, 53};
    for (int i = 16; i < 32; ++i) {
        const int j = i - 16;
        auto rm = [&](int o) { const int k = (j + o) & 15; return rotl64(M[k], k + 1); };
        const u64 add = ((rm(0) + rm(3) - rm(10) + u64(i) * 0x0555555555555555ULL) ^ H[(j + 7) & 15]);
        u64 s = add;
        if (i < 18) {  // expand1
            for (int k = 0; k < 16; ++k) s += bmw_s((k + 1) & 3, Q[j + k]);
        } else {  // expand2
            for (int k = 0; k < 14; ++k) s += (k & 1) ? rotl64(Q[j + k], kRot[k >> 1]) : Q[j + k];
            s += bmw_s(4, Q[i - 2]) + bmw_s(5, Q[i - 1]);
        }
        Q[i] = s;
    }
    u64 xl = 0, xh;
    for (int i = 16; i < 24; ++i) xl ^= Q[i];
    xh = xl;
    for (int i = 24; i < 32; ++i) xh ^= Q[i];
    // f2: shift amounts per output word (positive = left)
    static const int kXh[8] = {5, -7, -5, -1, -3, 6, -4, -11};
    static const int kQ[8] = {-5, 8, 5, 5, 0, -6, 6, 2};
    static const int kXl[8] = {8, -6, 6, 4, -3, -4, -7, -2};
    auto sh = [](u64 x, int s) { return s >= 0 ? x << s : x >> -s; };
    for (int i = 0; i < 8; ++i)
        out[i] = (sh(xh, kXh[i]) ^ sh(Q[16 + i], kQ[i]) ^ M[i]) + (xl ^ Q[24 + i] ^ Q[i]);
    for (int i = 8; i < 16; ++i)
        out[i] = rotl64(out[(i - 4) & 7], i + 1) + (xh ^ Q[16 + i] ^ M[i]) + (sh(xl, kXl[i - 8]) ^ (i == 8 ? Q[23] : Q[i + 7]) ^ Q[i]);
}

}  // namespace

Hash512 bmw512(const u8* data, size_t n) {
    u64 H[16], M[16], T[16];
    for (int i = 0; i < 16; ++i) {
        u64 v = 0;
        for (int b = 0; b < 8; ++b) v |= u64(0x80 + 8 * i + b) << (56 - 8 * b);
        H[i] = v;
    }
    const u64 bits = u64(n) * 8;
    for (; n >= 128; n -= 128, data += 128) {
        for (int i = 0; i < 16; ++i) M[i] = load_le64(data + 8 * i);
        bmw_compress(M, H, T);
        std::memcpy(H, T, sizeof H);
    }
    u8 buf[256] = {0};
    std::memcpy(buf, data, n);
    buf[n] = 0x80;
    const size_t len = n + 1 > 120 ? 256 : 128;
    store_le64(buf + len - 8, bits);
    for (size_t off = 0; off < len; off += 128) {
        for (int i = 0; i < 16; ++i) M[i] = load_le64(buf + off + 8 * i);
        bmw_compress(M, H, T);
        std::memcpy(H, T, sizeof H);
    }
    u64 F[16];
    for (int i = 0; i < 16; ++i) F[i] = 0xaaaaaaaaaaaaaaa0ULL + u64(i);
    bmw_compress(H, F, T);
    Hash512 out;
    for (int i = 0; i < 8; ++i) store_le64(out.bytes + 8 * i, T[8 + i]);
    return out;
}

}  // namespace nodexa
