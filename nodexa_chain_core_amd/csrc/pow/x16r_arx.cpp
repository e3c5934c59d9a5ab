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

Hash512 bmw512(const u8*, size_t) { throw std::runtime_error("bmw512: not implemented"); }

}  // namespace nodexa
