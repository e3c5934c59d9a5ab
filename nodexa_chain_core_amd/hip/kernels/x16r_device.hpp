// The seventeen X16R / X16RV2 primitives as per-lane device functions (hip/kernels/x16r.hip).
//
// Same constructions as the host's csrc/pow/x16r*.cpp (written from the SHA-3 round-2/3
// specifications, Whirlpool ISO/IEC 10118-3, Tiger 1995; parity with the sph_* family the
// reference links for HashX16R / HashX16RV2, src/hash.h:335-605), restated for one lane: fixed
// short inputs (the 80-byte header of the first step, a 64-byte digest after it), no heap, no
// statics, every derived table (AES S-box, Fugue / Whirlpool / Tiger tables, JH round-constant
// bits, Luffa / Hamsi / SIMD constants, CubeHash / Skein / Shabal IVs) read from x16r_tables.inc,
// which tools/x16r_gen_tables.cpp emits from the host code. Each primitive is the function of the
// slot, so a (step, slot) workgroup runs one of them with no divergence.
//
// The includer defines X16R_FN (the qualifiers of every function here: `__device__ inline` in the
// kernel, plain `inline` in the host-side self-check of tests/test_x16r_device.py) and includes
// <stdint.h>.
#pragma once

#include "x16r_tables.inc"

namespace x16rd {

typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;

struct H512 {
    u8 b[64];
};

X16R_FN u32 rl32(u32 x, int c) { c &= 31; return c ? (x << c) | (x >> (32 - c)) : x; }
X16R_FN u32 rr32(u32 x, int c) { c &= 31; return c ? (x >> c) | (x << (32 - c)) : x; }
X16R_FN u64 rl64(u64 x, int c) { c &= 63; return c ? (x << c) | (x >> (64 - c)) : x; }
X16R_FN u64 rr64(u64 x, int c) { c &= 63; return c ? (x >> c) | (x << (64 - c)) : x; }
X16R_FN u32 ld32(const u8* p) { return u32(p[0]) | (u32(p[1]) << 8) | (u32(p[2]) << 16) | (u32(p[3]) << 24); }
X16R_FN u64 ld64(const u8* p) { return u64(ld32(p)) | (u64(ld32(p + 4)) << 32); }
X16R_FN u32 ldb32(const u8* p) { return (u32(p[0]) << 24) | (u32(p[1]) << 16) | (u32(p[2]) << 8) | u32(p[3]); }
X16R_FN u64 ldb64(const u8* p) { return (u64(ldb32(p)) << 32) | u64(ldb32(p + 4)); }
X16R_FN void st32(u8* p, u32 v) { for (int i = 0; i < 4; ++i) p[i] = u8(v >> (8 * i)); }
X16R_FN void st64(u8* p, u64 v) { for (int i = 0; i < 8; ++i) p[i] = u8(v >> (8 * i)); }
X16R_FN void stb32(u8* p, u32 v) { for (int i = 0; i < 4; ++i) p[i] = u8(v >> (24 - 8 * i)); }
X16R_FN void stb64(u8* p, u64 v) { for (int i = 0; i < 8; ++i) p[i] = u8(v >> (56 - 8 * i)); }
X16R_FN void cpy(u8* d, const u8* s, int n) { for (int i = 0; i < n; ++i) d[i] = s[i]; }
X16R_FN void zero(u8* d, int n) { for (int i = 0; i < n; ++i) d[i] = 0; }
template <typename T>
X16R_FN void swp(T& a, T& b) { const T t = a; a = b; b = t; }

// ================================================================ BLAKE-512 (slot 0)
constexpr u64 kBlakeIV[8] = {0x6A09E667F3BCC908ULL, 0xBB67AE8584CAA73BULL, 0x3C6EF372FE94F82BULL, 0xA54FF53A5F1D36F1ULL,
                             0x510E527FADE682D1ULL, 0x9B05688C2B3E6C1FULL, 0x1F83D9ABFB41BD6BULL, 0x5BE0CD19137E2179ULL};
constexpr u64 kBlakeC[16] = {0x243F6A8885A308D3ULL, 0x13198A2E03707344ULL, 0xA4093822299F31D0ULL, 0x082EFA98EC4E6C89ULL,
                             0x452821E638D01377ULL, 0xBE5466CF34E90C6CULL, 0xC0AC29B7C97C50DDULL, 0x3F84D5B5B5470917ULL,
                             0x9216D5D98979FB1BULL, 0xD1310BA698DFB5ACULL, 0x2FFD72DBD01ADFB7ULL, 0xB8E1AFED6A267E96ULL,
                             0xBA7C9045F12C7F99ULL, 0x24A19947B3916CF7ULL, 0x0801F2E2858EFC16ULL, 0x636920D871574E69ULL};
constexpr u8 kSigma[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

X16R_FN void blake_g(u64* v, const u64* m, int r, int i, int a, int b, int c, int d) {
    const u8* s = kSigma[r % 10];
    v[a] = v[a] + v[b] + (m[s[2 * i]] ^ kBlakeC[s[2 * i + 1]]);
    v[d] = rr64(v[d] ^ v[a], 32);
    v[c] = v[c] + v[d];
    v[b] = rr64(v[b] ^ v[c], 25);
    v[a] = v[a] + v[b] + (m[s[2 * i + 1]] ^ kBlakeC[s[2 * i]]);
    v[d] = rr64(v[d] ^ v[a], 16);
    v[c] = v[c] + v[d];
    v[b] = rr64(v[b] ^ v[c], 11);
}

X16R_FN void blake_compress(u64 h[8], const u8* block, u64 t0) {
    u64 m[16], v[16];
    for (int i = 0; i < 16; ++i) m[i] = ldb64(block + 8 * i);
    for (int i = 0; i < 8; ++i) v[i] = h[i];
    v[8] = kBlakeC[0]; v[9] = kBlakeC[1]; v[10] = kBlakeC[2]; v[11] = kBlakeC[3];
    v[12] = t0 ^ kBlakeC[4]; v[13] = t0 ^ kBlakeC[5]; v[14] = kBlakeC[6]; v[15] = kBlakeC[7];
    for (int r = 0; r < 16; ++r) {
        blake_g(v, m, r, 0, 0, 4, 8, 12); blake_g(v, m, r, 1, 1, 5, 9, 13);
        blake_g(v, m, r, 2, 2, 6, 10, 14); blake_g(v, m, r, 3, 3, 7, 11, 15);
        blake_g(v, m, r, 4, 0, 5, 10, 15); blake_g(v, m, r, 5, 1, 6, 11, 12);
        blake_g(v, m, r, 6, 2, 7, 8, 13); blake_g(v, m, r, 7, 3, 4, 9, 14);
    }
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

X16R_FN void blake512(const u8* data, int n, u8* out) {  // n < 112: one padded block
    u64 h[8];
    for (int i = 0; i < 8; ++i) h[i] = kBlakeIV[i];
    u8 buf[128];
    zero(buf, 128);
    cpy(buf, data, n);
    buf[n] = 0x80;
    buf[111] |= 0x01;
    const u64 bits = u64(n) * 8;
    stb64(buf + 120, bits);
    blake_compress(h, buf, n ? bits : 0);
    for (int i = 0; i < 8; ++i) stb64(out + 8 * i, h[i]);
}

// ================================================================ BMW-512 (slot 1)
struct BmwW {
    int idx[5];
    int sgn[5];
};
constexpr BmwW kBmwW[16] = {
    {{5, 7, 10, 13, 14}, {1, -1, 1, 1, 1}},  {{6, 8, 11, 14, 15}, {1, -1, 1, 1, -1}},
    {{0, 7, 9, 12, 15}, {1, 1, 1, -1, 1}},   {{0, 1, 8, 10, 13}, {1, -1, 1, -1, 1}},
    {{1, 2, 9, 11, 14}, {1, 1, 1, -1, -1}},  {{3, 2, 10, 12, 15}, {1, -1, 1, -1, 1}},
    {{4, 0, 3, 11, 13}, {1, -1, -1, -1, 1}}, {{1, 4, 5, 12, 14}, {1, -1, -1, -1, -1}},
    {{2, 5, 6, 13, 15}, {1, -1, -1, 1, -1}}, {{0, 3, 6, 7, 14}, {1, -1, 1, -1, 1}},
    {{8, 1, 4, 7, 15}, {1, -1, -1, -1, 1}},  {{8, 0, 2, 5, 9}, {1, -1, -1, -1, 1}},
    {{1, 3, 6, 9, 10}, {1, 1, -1, -1, 1}},   {{2, 4, 7, 10, 11}, {1, 1, 1, 1, 1}},
    {{3, 5, 8, 11, 12}, {1, -1, 1, -1, -1}}, {{12, 4, 6, 9, 13}, {1, -1, -1, -1, 1}}};
constexpr int kBmwRot[7] = {5, 11, 27, 32, 37, 43, 53};
constexpr int kBmwXh[8] = {5, -7, -5, -1, -3, 6, -4, -11};
constexpr int kBmwQ[8] = {-5, 8, 5, 5, 0, -6, 6, 2};
constexpr int kBmwXl[8] = {8, -6, 6, 4, -3, -4, -7, -2};

X16R_FN u64 bmw_s(int k, u64 x) {
    switch (k) {
        case 0: return (x >> 1) ^ (x << 3) ^ rl64(x, 4) ^ rl64(x, 37);
        case 1: return (x >> 1) ^ (x << 2) ^ rl64(x, 13) ^ rl64(x, 43);
        case 2: return (x >> 2) ^ (x << 1) ^ rl64(x, 19) ^ rl64(x, 53);
        case 3: return (x >> 2) ^ (x << 2) ^ rl64(x, 28) ^ rl64(x, 59);
        case 4: return (x >> 1) ^ x;
        default: return (x >> 2) ^ x;
    }
}
X16R_FN u64 bmw_sh(u64 x, int s) { return s >= 0 ? x << s : x >> -s; }

X16R_FN void bmw_compress(const u64 M[16], const u64 H[16], u64 out[16]) {
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
    for (int i = 16; i < 32; ++i) {
        const int j = i - 16;
        const int k0 = j & 15, k3 = (j + 3) & 15, k10 = (j + 10) & 15;
        const u64 add = ((rl64(M[k0], k0 + 1) + rl64(M[k3], k3 + 1) - rl64(M[k10], k10 + 1) +
                          u64(i) * 0x0555555555555555ULL) ^ H[(j + 7) & 15]);
        u64 s = add;
        if (i < 18) {
            for (int k = 0; k < 16; ++k) s += bmw_s((k + 1) & 3, Q[j + k]);
        } else {
            for (int k = 0; k < 14; ++k) s += (k & 1) ? rl64(Q[j + k], kBmwRot[k >> 1]) : Q[j + k];
            s += bmw_s(4, Q[i - 2]) + bmw_s(5, Q[i - 1]);
        }
        Q[i] = s;
    }
    u64 xl = 0, xh;
    for (int i = 16; i < 24; ++i) xl ^= Q[i];
    xh = xl;
    for (int i = 24; i < 32; ++i) xh ^= Q[i];
    for (int i = 0; i < 8; ++i)
        out[i] = (bmw_sh(xh, kBmwXh[i]) ^ bmw_sh(Q[16 + i], kBmwQ[i]) ^ M[i]) + (xl ^ Q[24 + i] ^ Q[i]);
    for (int i = 8; i < 16; ++i)
        out[i] = rl64(out[(i - 4) & 7], i + 1) + (xh ^ Q[16 + i] ^ M[i]) +
                 (bmw_sh(xl, kBmwXl[i - 8]) ^ (i == 8 ? Q[23] : Q[i + 7]) ^ Q[i]);
}

X16R_FN void bmw512(const u8* data, int n, u8* out) {  // n < 120: one padded block
    u64 H[16], M[16], T[16];
    for (int i = 0; i < 16; ++i) {
        u64 v = 0;
        for (int b = 0; b < 8; ++b) v |= u64(0x80 + 8 * i + b) << (56 - 8 * b);
        H[i] = v;
    }
    u8 buf[128];
    zero(buf, 128);
    cpy(buf, data, n);
    buf[n] = 0x80;
    st64(buf + 120, u64(n) * 8);
    for (int i = 0; i < 16; ++i) M[i] = ld64(buf + 8 * i);
    bmw_compress(M, H, T);
    u64 F[16];
    for (int i = 0; i < 16; ++i) F[i] = 0xaaaaaaaaaaaaaaa0ULL + u64(i);
    bmw_compress(T, F, H);
    for (int i = 0; i < 8; ++i) st64(out + 8 * i, H[8 + i]);
}

// ================================================================ AES round
// The round on four little-endian column words through 4 x 256 u32 tables (kX16rAesT).
X16R_FN void aes_round_w(u32 x[4], u32 k0, u32 k1, const u32* T) {
    const u32 y0 = T[x[0] & 0xFF] ^ T[256 + ((x[1] >> 8) & 0xFF)] ^ T[512 + ((x[2] >> 16) & 0xFF)] ^ T[768 + (x[3] >> 24)];
    const u32 y1 = T[x[1] & 0xFF] ^ T[256 + ((x[2] >> 8) & 0xFF)] ^ T[512 + ((x[3] >> 16) & 0xFF)] ^ T[768 + (x[0] >> 24)];
    const u32 y2 = T[x[2] & 0xFF] ^ T[256 + ((x[3] >> 8) & 0xFF)] ^ T[512 + ((x[0] >> 16) & 0xFF)] ^ T[768 + (x[1] >> 24)];
    const u32 y3 = T[x[3] & 0xFF] ^ T[256 + ((x[0] >> 8) & 0xFF)] ^ T[512 + ((x[1] >> 16) & 0xFF)] ^ T[768 + (x[2] >> 24)];
    x[0] = y0 ^ k0;
    x[1] = y1 ^ k1;
    x[2] = y2;
    x[3] = y3;
}
X16R_FN u32 xtime4(u32 v) { return ((v & 0x7F7F7F7Fu) << 1) ^ (((v >> 7) & 0x01010101u) * 0x1Bu); }

// ================================================================ Groestl-512 (slot 2)
// 16 u64 columns (row i in byte i); SubBytes + ShiftBytes + MixBytes as 8 table lookups per column.
constexpr int kGrShiftP[8] = {0, 1, 2, 3, 4, 5, 6, 11};
constexpr int kGrShiftQ[8] = {1, 3, 5, 11, 0, 2, 4, 6};

X16R_FN void groestl_perm(u64 st[16], bool q, const u64* T) {
    const int* sh = q ? kGrShiftQ : kGrShiftP;
    u64 t[16];
    for (int r = 0; r < 14; ++r) {
        for (int j = 0; j < 16; ++j) st[j] ^= q ? ~(u64((j << 4) ^ r) << 56) : u64((j << 4) ^ r);
        for (int j = 0; j < 16; ++j) {
            u64 v = 0;
            for (int k = 0; k < 8; ++k) v ^= T[256 * k + u8(st[(j + sh[k]) & 15] >> (8 * k))];
            t[j] = v;
        }
        for (int j = 0; j < 16; ++j) st[j] = t[j];
    }
}

X16R_FN void groestl512(const u8* data, int n, u8* out, const u64* T = kX16rGroestlT) {  // n < 120: one block
    u8 buf[128];
    zero(buf, 128);
    cpy(buf, data, n);
    buf[n] = 0x80;
    stb64(buf + 120, 1);
    u64 h[16], p[16], q[16];
    for (int j = 0; j < 16; ++j) {
        h[j] = j == 15 ? (u64(0x02) << 48) : 0;
        q[j] = ld64(buf + 8 * j);
        p[j] = h[j] ^ q[j];
    }
    groestl_perm(p, false, T);
    groestl_perm(q, true, T);
    for (int j = 0; j < 16; ++j) {
        h[j] ^= p[j] ^ q[j];
        p[j] = h[j];
    }
    groestl_perm(p, false, T);
    for (int j = 0; j < 8; ++j) st64(out + 8 * j, p[8 + j] ^ h[8 + j]);
}

// ================================================================ JH-512 (slot 3)
// Bit-sliced E8 over eight 128-bit words (csrc/pow/x16r_bitslice.cpp derives the form and the
// per-round constant masks kX16rJhC from the element-form specification).
X16R_FN void jh_sbox(u64& m0, u64& m1, u64& m2, u64& m3, u64 cc) {
    m3 = ~m3;
    m0 ^= ~m2 & cc;
    const u64 t0 = cc ^ (m0 & m1);
    m0 ^= m2 & m3;
    m3 ^= ~m1 & m2;
    m1 ^= m0 & m2;
    m2 ^= m0 & ~m3;
    m0 ^= m1 | m3;
    m3 ^= m1 & m2;
    m1 ^= t0 & m0;
    m2 ^= t0;
}
constexpr u64 kJhSwapMask[6] = {0x5555555555555555ULL, 0x3333333333333333ULL, 0x0F0F0F0F0F0F0F0FULL,
                                0x00FF00FF00FF00FFULL, 0x0000FFFF0000FFFFULL, 0x00000000FFFFFFFFULL};

X16R_FN void jh_e8(u8 H[128]) {
    u64 x[8][2];
    for (int j = 0; j < 8; ++j) {
        x[j][0] = ld64(H + 16 * j);
        x[j][1] = ld64(H + 16 * j + 8);
    }
    for (int r = 0; r < 42; ++r) {
        for (int g = 0; g < 2; ++g)
            for (int h = 0; h < 2; ++h) jh_sbox(x[g][h], x[2 + g][h], x[4 + g][h], x[6 + g][h], kX16rJhC[4 * r + 2 * g + h]);
        for (int h = 0; h < 2; ++h) {
            x[1][h] ^= x[2][h];
            x[3][h] ^= x[4][h];
            x[5][h] ^= x[6][h] ^ x[0][h];
            x[7][h] ^= x[0][h];
            x[0][h] ^= x[3][h];
            x[2][h] ^= x[5][h];
            x[4][h] ^= x[7][h] ^ x[1][h];
            x[6][h] ^= x[1][h];
        }
        const int k = r % 7;
        for (int j = 1; j < 8; j += 2) {
            if (k == 6) {
                swp(x[j][0], x[j][1]);
            } else {
                const int sh = 1 << k;
                const u64 m = kJhSwapMask[k];
                for (int h = 0; h < 2; ++h) x[j][h] = ((x[j][h] & m) << sh) | ((x[j][h] >> sh) & m);
            }
        }
    }
    for (int j = 0; j < 8; ++j) {
        st64(H + 16 * j, x[j][0]);
        st64(H + 16 * j + 8, x[j][1]);
    }
}

X16R_FN void jh_f8(u8 H[128], const u8 m[64]) {
    for (int i = 0; i < 64; ++i) H[i] ^= m[i];
    jh_e8(H);
    for (int i = 0; i < 64; ++i) H[64 + i] ^= m[i];
}

X16R_FN void jh512(const u8* data, int n, u8* out) {  // 0 < n < 128
    u8 H[128];
    cpy(H, kX16rJhIv, 128);
    const u64 bits = u64(n) * 8;
    for (; n >= 64; n -= 64, data += 64) jh_f8(H, data);
    u8 buf[128];
    zero(buf, 128);
    cpy(buf, data, n);
    buf[n] = 0x80;
    const int len = n == 0 ? 64 : 128;
    stb64(buf + len - 8, bits);
    jh_f8(H, buf);
    if (len == 128) jh_f8(H, buf + 64);
    cpy(out, H + 64, 64);
}

// ================================================================ Keccak-512 (slot 4)
constexpr u64 kKeccakRc[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL, 0x000000000000808bULL,
    0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL, 0x000000000000008aULL, 0x0000000000000088ULL,
    0x0000000080008009ULL, 0x000000008000000aULL, 0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL,
    0x8000000000008003ULL, 0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
constexpr int kKeccakRho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

X16R_FN void keccak_f(u64 a[25]) {
    for (int round = 0; round < 24; ++round) {
        u64 c[5], b[25];
        for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
        for (int x = 0; x < 5; ++x) {
            const u64 d = c[(x + 4) % 5] ^ rl64(c[(x + 1) % 5], 1);
            for (int y = 0; y < 5; ++y) a[x + 5 * y] ^= d;
        }
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = rl64(a[x + 5 * y], kKeccakRho[x + 5 * y]);
        for (int y = 0; y < 5; ++y)
            for (int x = 0; x < 5; ++x) a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
        a[0] ^= kKeccakRc[round];
    }
}

X16R_FN void keccak512(const u8* data, int n, u8* out) {  // rate 72, original 0x01 padding
    u64 st[25];
    for (int i = 0; i < 25; ++i) st[i] = 0;
    for (; n >= 72; n -= 72, data += 72) {
        for (int i = 0; i < 9; ++i) st[i] ^= ld64(data + 8 * i);
        keccak_f(st);
    }
    u8 last[72];
    zero(last, 72);
    cpy(last, data, n);
    last[n] ^= 0x01;
    last[71] ^= 0x80;
    for (int i = 0; i < 9; ++i) st[i] ^= ld64(last + 8 * i);
    keccak_f(st);
    for (int i = 0; i < 8; ++i) st64(out + 8 * i, st[i]);
}

// ================================================================ Skein-512-512 (slot 5)
constexpr int kSkeinRot[8][4] = {{46, 36, 19, 37}, {33, 27, 14, 42}, {17, 49, 36, 39}, {44, 9, 54, 56},
                                 {39, 30, 34, 24}, {13, 50, 10, 17}, {25, 29, 39, 43}, {8, 35, 56, 22}};
constexpr int kSkeinPerm[8] = {2, 1, 4, 7, 6, 5, 0, 3};

X16R_FN void threefish512(const u64 key[8], const u64 tweak[2], const u64 in[8], u64 out[8]) {
    u64 k[9], t[3] = {tweak[0], tweak[1], tweak[0] ^ tweak[1]};
    k[8] = 0x1BD11BDAA9FC1A22ULL;
    for (int i = 0; i < 8; ++i) { k[i] = key[i]; k[8] ^= key[i]; }
    u64 v[8];
    for (int i = 0; i < 8; ++i) v[i] = in[i];
    for (int s = 0; s <= 18; ++s) {
        for (int i = 0; i < 8; ++i) v[i] += k[(s + i) % 9];
        v[5] += t[s % 3];
        v[6] += t[(s + 1) % 3];
        v[7] += u64(s);
        if (s == 18) break;
        for (int d = 4 * s; d < 4 * s + 4; ++d) {
            for (int j = 0; j < 4; ++j) {
                v[2 * j] += v[2 * j + 1];
                v[2 * j + 1] = rl64(v[2 * j + 1], kSkeinRot[d % 8][j]) ^ v[2 * j];
            }
            u64 p[8];
            for (int i = 0; i < 8; ++i) p[i] = v[kSkeinPerm[i]];
            for (int i = 0; i < 8; ++i) v[i] = p[i];
        }
    }
    for (int i = 0; i < 8; ++i) out[i] = v[i];
}

X16R_FN void skein_ubi(u64 g[8], const u8* m, int n, u64 type) {
    u64 pos = 0;
    bool first = true;
    do {
        const int take = n > 64 ? 64 : n;
        u8 blk[64];
        zero(blk, 64);
        cpy(blk, m, take);
        pos += u64(take);
        m += take;
        n -= take;
        const bool fin = n == 0;
        const u64 tw[2] = {pos, (type << 56) | (u64(first) << 62) | (u64(fin) << 63)};
        u64 w[8], e[8];
        for (int i = 0; i < 8; ++i) w[i] = ld64(blk + 8 * i);
        threefish512(g, tw, w, e);
        for (int i = 0; i < 8; ++i) g[i] = e[i] ^ w[i];
        first = false;
    } while (n > 0);
}

X16R_FN void skein512(const u8* data, int n, u8* out) {
    u64 g[8];
    for (int i = 0; i < 8; ++i) g[i] = kX16rSkeinIv[i];
    skein_ubi(g, data, n, 48);
    u8 ctr[8];
    zero(ctr, 8);
    skein_ubi(g, ctr, 8, 63);
    for (int i = 0; i < 8; ++i) st64(out + 8 * i, g[i]);
}

// ================================================================ Luffa-512 (slot 6)
X16R_FN void luffa_x2(u32 d[8], const u32 s[8]) {
    const u32 t = s[7];
    const u32 r[8] = {t, s[0] ^ t, s[1], s[2] ^ t, s[3] ^ t, s[4], s[5], s[6]};
    for (int i = 0; i < 8; ++i) d[i] = r[i];
}
X16R_FN void luffa_xor(u32 d[8], const u32 a[8], const u32 b[8]) {
    for (int i = 0; i < 8; ++i) d[i] = a[i] ^ b[i];
}
X16R_FN void sub_crumb(u32& a0, u32& a1, u32& a2, u32& a3) {
    u32 t = a0;
    a0 |= a1; a2 ^= a3; a1 = ~a1; a0 ^= a3; a3 &= t; a1 ^= a3; a3 ^= a2; a2 &= a0;
    a0 = ~a0; a2 ^= a1; a1 |= a3; t ^= a1; a3 ^= a2; a2 &= a1; a1 ^= a0; a0 = t;
}
X16R_FN void mix_word(u32& u, u32& v) {
    v ^= u;
    u = rl32(u, 2) ^ v;
    v = rl32(v, 14) ^ u;
    u = rl32(u, 10) ^ v;
    v = rl32(v, 1);
}

X16R_FN void luffa_round(u32 V[5][8], const u8 blk[32]) {
    u32 M[8], a[8], b[8];
    for (int i = 0; i < 8; ++i) M[i] = ldb32(blk + 4 * i);
    luffa_xor(a, V[0], V[1]);
    luffa_xor(b, V[2], V[3]);
    luffa_xor(a, a, b);
    luffa_xor(a, a, V[4]);
    luffa_x2(a, a);
    for (int j = 0; j < 5; ++j) luffa_xor(V[j], V[j], a);
    luffa_x2(b, V[0]);
    luffa_xor(b, b, V[1]);
    for (int j = 1; j < 4; ++j) { luffa_x2(V[j], V[j]); luffa_xor(V[j], V[j], V[j + 1]); }
    luffa_x2(V[4], V[4]);
    luffa_xor(V[4], V[4], V[0]);
    luffa_x2(V[0], b);
    luffa_xor(V[0], V[0], V[4]);
    for (int j = 4; j > 1; --j) { luffa_x2(V[j], V[j]); luffa_xor(V[j], V[j], V[j - 1]); }
    luffa_x2(V[1], V[1]);
    luffa_xor(V[1], V[1], b);
    for (int j = 0; j < 5; ++j) {
        if (j) luffa_x2(M, M);
        luffa_xor(V[j], V[j], M);
    }
    for (int j = 0; j < 5; ++j) {
        u32* x = V[j];
        for (int i = 4; i < 8; ++i) x[i] = rl32(x[i], j);
        for (int r = 0; r < 8; ++r) {
            sub_crumb(x[0], x[1], x[2], x[3]);
            sub_crumb(x[5], x[6], x[7], x[4]);
            for (int i = 0; i < 4; ++i) mix_word(x[i], x[i + 4]);
            x[0] ^= kX16rLuffaRc[16 * j + r];
            x[4] ^= kX16rLuffaRc[16 * j + 8 + r];
        }
    }
}

X16R_FN void luffa512(const u8* data, int n, u8* out) {
    u32 V[5][8];
    for (int j = 0; j < 5; ++j)
        for (int i = 0; i < 8; ++i) V[j][i] = kX16rLuffaIv[8 * j + i];
    for (; n >= 32; n -= 32, data += 32) luffa_round(V, data);
    u8 buf[32];
    zero(buf, 32);
    cpy(buf, data, n);
    buf[n] = 0x80;
    luffa_round(V, buf);
    zero(buf, 32);
    for (int half = 0; half < 2; ++half) {
        luffa_round(V, buf);
        for (int i = 0; i < 8; ++i) stb32(out + 32 * half + 4 * i, V[0][i] ^ V[1][i] ^ V[2][i] ^ V[3][i] ^ V[4][i]);
    }
}

// ================================================================ CubeHash16/32-512 (slot 7)
X16R_FN void cubehash_rounds(u32 x[32], int rounds) {
    for (int r = 0; r < rounds; ++r) {
        for (int j = 0; j < 16; ++j) x[16 + j] += x[j];
        for (int j = 0; j < 16; ++j) x[j] = rl32(x[j], 7);
        for (int j = 0; j < 8; ++j) swp(x[j], x[j + 8]);
        for (int j = 0; j < 16; ++j) x[j] ^= x[16 + j];
        for (int j = 16; j < 32; ++j)
            if (!(j & 2)) swp(x[j], x[j + 2]);
        for (int j = 0; j < 16; ++j) x[16 + j] += x[j];
        for (int j = 0; j < 16; ++j) x[j] = rl32(x[j], 11);
        for (int j = 0; j < 16; ++j)
            if (!(j & 4)) swp(x[j], x[j + 4]);
        for (int j = 0; j < 16; ++j) x[j] ^= x[16 + j];
        for (int j = 16; j < 32; j += 2) swp(x[j], x[j + 1]);
    }
}

X16R_FN void cubehash512(const u8* data, int n, u8* out) {
    u32 x[32];
    for (int i = 0; i < 32; ++i) x[i] = kX16rCubeIv[i];
    for (; n >= 32; n -= 32, data += 32) {
        for (int i = 0; i < 8; ++i) x[i] ^= ld32(data + 4 * i);
        cubehash_rounds(x, 16);
    }
    u8 last[32];
    zero(last, 32);
    cpy(last, data, n);
    last[n] = 0x80;
    for (int i = 0; i < 8; ++i) x[i] ^= ld32(last + 4 * i);
    cubehash_rounds(x, 16);
    x[31] ^= 1;
    cubehash_rounds(x, 160);
    for (int i = 0; i < 16; ++i) st32(out + 4 * i, x[i]);
}

// ================================================================ SHAvite-3-512 (slot 8)
X16R_FN void aes_words(u32 x[4], const u32* T) { aes_round_w(x, 0, 0, T); }

X16R_FN void shavite_inject(u32* rk, int u, const u32 cnt[4], int a, int b, int c, int d) {
    rk[u] ^= cnt[a]; rk[u + 1] ^= cnt[b]; rk[u + 2] ^= cnt[c]; rk[u + 3] ^= ~cnt[d];
}

X16R_FN void shavite_F(u32 L[4], const u32 R[4], const u32* rk, int& r_idx, const u32* sbox) {
    u32 x[4];
    for (int k = 0; k < 4; ++k) x[k] = R[k] ^ rk[r_idx++];
    aes_words(x, sbox);
    for (int j = 0; j < 3; ++j) {
        for (int k = 0; k < 4; ++k) x[k] ^= rk[r_idx++];
        aes_words(x, sbox);
    }
    for (int k = 0; k < 4; ++k) L[k] ^= x[k];
}

X16R_FN void shavite_c512(u32 h[16], const u8 msg[128], const u32 cnt[4], const u32* sbox) {
    u32 rk[448];
    for (int i = 0; i < 32; ++i) rk[i] = ld32(msg + 4 * i);
    int u = 32;
    for (;;) {
        for (int s = 0; s < 8; ++s) {
            u32 x[4] = {rk[u - 31], rk[u - 30], rk[u - 29], rk[u - 32]};
            aes_words(x, sbox);
            for (int k = 0; k < 4; ++k) rk[u + k] = x[k] ^ rk[u - 4 + k];
            if (u == 32) shavite_inject(rk, 32, cnt, 0, 1, 2, 3);
            else if (u == 164) shavite_inject(rk, 164, cnt, 3, 2, 1, 0);
            else if (u == 316) shavite_inject(rk, 316, cnt, 2, 3, 0, 1);
            else if (u == 440) shavite_inject(rk, 440, cnt, 1, 0, 3, 2);
            u += 4;
        }
        if (u == 448) break;
        for (int s = 0; s < 8; ++s, u += 4)
            for (int k = 0; k < 4; ++k) rk[u + k] = rk[u - 32 + k] ^ rk[u - 7 + k];
    }
    u32 P[4][4];
    for (int b = 0; b < 4; ++b)
        for (int k = 0; k < 4; ++k) P[b][k] = h[4 * b + k];
    int r_idx = 0;
    for (int r = 0; r < 14; ++r) {
        shavite_F(P[0], P[1], rk, r_idx, sbox);
        shavite_F(P[2], P[3], rk, r_idx, sbox);
        u32 t[4];
        for (int k = 0; k < 4; ++k) {
            t[k] = P[3][k];
            P[3][k] = P[2][k];
            P[2][k] = P[1][k];
            P[1][k] = P[0][k];
            P[0][k] = t[k];
        }
    }
    for (int b = 0; b < 4; ++b)
        for (int k = 0; k < 4; ++k) h[4 * b + k] ^= P[b][k];
}

constexpr u32 kShaviteIV[16] = {0x72FCCDD8, 0x79CA4727, 0x128A077B, 0x40D55AEC, 0xD1901A06, 0x430AE307,
                                0xB29F5CD1, 0xDF07FBFC, 0x8E45D73D, 0x681AB538, 0xBDE86578, 0xDD577E47,
                                0xE275EADE, 0x502D9FCD, 0xB9357178, 0x022A4B9A};

X16R_FN void shavite512(const u8* data, int n, u8* out, const u32* sbox = kX16rAesT) {  // 0 < n < 110
    u32 h[16];
    for (int i = 0; i < 16; ++i) h[i] = kShaviteIV[i];
    const u64 bits = u64(n) * 8;
    u8 buf[128];
    zero(buf, 128);
    cpy(buf, data, n);
    buf[n] = 0x80;
    const u32 total[4] = {u32(bits), u32(bits >> 32), 0, 0};
    for (int i = 0; i < 4; ++i) st32(buf + 110 + 4 * i, total[i]);
    buf[126] = 0x00;
    buf[127] = 0x02;
    shavite_c512(h, buf, total, sbox);
    for (int i = 0; i < 16; ++i) st32(out + 4 * i, h[i]);
}

// ================================================================ SIMD-512 (slot 9)
constexpr int kSimdSb[4][8] = {{4, 6, 0, 2, 7, 5, 3, 1}, {15, 11, 12, 8, 9, 13, 10, 14},
                               {17, 18, 23, 20, 22, 21, 16, 19}, {30, 24, 25, 31, 27, 29, 28, 26}};
constexpr int kSimdRot[4][4] = {{3, 23, 17, 27}, {28, 19, 22, 7}, {29, 9, 15, 5}, {4, 13, 10, 25}};
constexpr int kSimdPerm[7] = {1, 6, 2, 3, 5, 7, 4};
constexpr int kSimdFf[4][3] = {{4, 13, 4}, {13, 10, 5}, {10, 25, 6}, {25, 4, 0}};
constexpr u32 kSimdIV[32] = {
    0x0BA16B95, 0x72F999AD, 0x9FECC2AE, 0xBA3264FC, 0x5E894929, 0x8E9F30E5, 0x2F1DAA37, 0xF0F2C558,
    0xAC506643, 0xA90635A5, 0xE25B878B, 0xAAB7878F, 0x88817F7A, 0x0A02892B, 0x559A7550, 0x598F657E,
    0x7EEF60A1, 0x6B70E3E8, 0x9C1714D1, 0xB958E2A8, 0xAB02675E, 0xED1C014F, 0xCD8D65BB, 0xFDB7A257,
    0x09254899, 0xD699C7BC, 0x9019B6DC, 0x2B9022E4, 0x8FA14956, 0x21BF9BD3, 0xB94D0943, 0x6FFDDC22};

// x mod 257 for 0 <= x <= 2^16 (every use here): 256 = -1 (mod 257), so x = 256 h + l = l - h.
X16R_FN int mod257(int x) {
    int r = (x & 255) - (x >> 8);
    r += r < 0 ? 257 : 0;
    return r >= 257 ? r - 257 : r;
}

X16R_FN u32 simd_inner(int lo, int hi, int mm) { return (u32(lo * mm) & 0xFFFFu) + (u32(hi * mm) << 16); }

X16R_FN void simd_step(u32 A[8], u32 B[8], u32 C[8], u32 D[8], const u32 w[8], int f, int r, int s, int pc) {
    u32 tA[8];
    for (int n = 0; n < 8; ++n) tA[n] = rl32(A[n], r);
    for (int n = 0; n < 8; ++n) {
        const u32 fv = f ? ((A[n] & B[n]) | ((A[n] | B[n]) & C[n])) : (((B[n] ^ C[n]) & A[n]) ^ C[n]);
        const u32 tt = D[n] + w[n] + fv;
        A[n] = rl32(tt, s) + tA[n ^ pc];
        D[n] = C[n];
        C[n] = B[n];
        B[n] = tA[n];
    }
}

// The expanded message: element i of the 256-entry NTT buffer `qb` spaced `qs` apart (the kernel
// interleaves the buffers of a workgroup's lanes in LDS; the host self-check uses a local array,
// qs = 1).
#ifndef SIMD_NTT_BATCH
#define SIMD_NTT_BATCH 8
#endif
// `n64`: only bytes 0..63 of the block can be nonzero (a 64-byte input's message block). Their
// bit-reversed positions are the multiples of 4, so the first two butterfly stages only copy each
// of them over its group of four: the NTT starts at the third stage.
X16R_FN void simd_expand(const u8 blk[128], bool last, int16_t* qb, int qs, const int16_t* pw, const int16_t* yn,
                         const int16_t* yf, bool n64 = false) {
#define Q(i) qb[(i) * qs]
    // 256-point NTT over Z_257 (root 41), radix 2, bit-reversed input
    int len = 2;
    if (n64) {
        for (int j = 0; j < 64; ++j) {
            int r = 0;
            for (int b = 0; b < 6; ++b) r |= ((j >> b) & 1) << (7 - b);
            const int16_t v = int16_t(blk[j]);
            Q(r) = v;
            Q(r + 1) = v;
            Q(r + 2) = v;
            Q(r + 3) = v;
        }
        len = 8;
    } else {
        for (int j = 0; j < 256; ++j) {
            int r = 0;
            for (int b = 0; b < 8; ++b) r |= ((j >> b) & 1) << (7 - b);
            Q(r) = int16_t(j < 128 ? int(blk[j]) : 0);
        }
    }
    // a stage's 128 butterflies are independent: SIMD_NTT_BATCH of them at a time, every load before
    // any store, so that many LDS round trips are in flight at once (one lane's NTT is otherwise a
    // chain of dependent LDS accesses, and a step runs one wave per SIMD: nothing hides them)
    for (; len <= 256; len <<= 1) {
        const int half = len / 2, lg = __builtin_ctz(unsigned(half)), stride = 256 / len;
        for (int b0 = 0; b0 < 128; b0 += SIMD_NTT_BATCH) {
            int lo[SIMD_NTT_BATCH], u[SIMD_NTT_BATCH], v[SIMD_NTT_BATCH];
#pragma unroll
            for (int t = 0; t < SIMD_NTT_BATCH; ++t) {
                const int b = b0 + t, k = b & (half - 1);
                lo[t] = ((b >> lg) << (lg + 1)) + k;
                u[t] = Q(lo[t]);
                v[t] = Q(lo[t] + half) * pw[stride * k];
            }
#pragma unroll
            for (int t = 0; t < SIMD_NTT_BATCH; ++t) {
                const int w = mod257(v[t]);
                Q(lo[t]) = int16_t(mod257(u[t] + w));
                Q(lo[t] + half) = int16_t(mod257(u[t] - w + 257));
            }
        }
    }
    const int16_t* yoff = last ? yf : yn;
    for (int i = 0; i < 256; ++i) {
        const int acc = mod257(Q(i) + yoff[i]);
        Q(i) = int16_t(acc <= 128 ? acc : acc - 257);
    }
#undef Q
}

// The four rounds and the feed-forward; q(i) returns expanded-message element i. For the final
// block of a 64-byte input q reads its constant expansion (kX16rSimdFin64, made by the host,
// x16r_simd.cpp): with the rounds unrolled every message word is then a literal.
template <class QF>
X16R_FN __attribute__((always_inline)) void simd_rounds(u32 state[32], const u8 blk[128], QF q) {
    u32 A[8], B[8], C[8], D[8], saved[32];
    for (int i = 0; i < 32; ++i) saved[i] = state[i];
    for (int i = 0; i < 8; ++i) {
        A[i] = state[i] ^ ld32(blk + 4 * i);
        B[i] = state[8 + i] ^ ld32(blk + 32 + 4 * i);
        C[i] = state[16 + i] ^ ld32(blk + 64 + 4 * i);
        D[i] = state[24 + i] ^ ld32(blk + 96 + 4 * i);
    }
    // unrolled: the step's lane permutation n ^ pc and rotations become constants (a runtime
    // pc would index tA[] through scratch memory on the GPU)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int sb = kSimdSb[r][j];
            u32 w[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (r < 2) {
                    w[k] = simd_inner(q(16 * sb + 2 * k), q(16 * sb + 2 * k + 1), 185);
                } else {
                    const int base = 16 * (sb - 8 * r) + 2 * k + (r == 3 ? 1 : 0);
                    w[k] = simd_inner(q(base), q(base + 128), 233);
                }
            }
            simd_step(A, B, C, D, w, j >= 4, kSimdRot[r][j & 3], kSimdRot[r][(j + 1) & 3], kSimdPerm[(j + r) % 7]);
        }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        simd_step(A, B, C, D, saved + 8 * k, 0, kSimdFf[k][0], kSimdFf[k][1], kSimdPerm[kSimdFf[k][2]]);
    for (int i = 0; i < 8; ++i) {
        state[i] = A[i];
        state[8 + i] = B[i];
        state[16 + i] = C[i];
        state[24 + i] = D[i];
    }
}

struct SimdQBuf {  // the expansion in the NTT buffer
    const int16_t* qb;
    int qs;
    X16R_FN int operator()(int i) const { return qb[i * qs]; }
};
struct SimdQFin64 {  // the constant expansion of a 64-byte input's final block
    X16R_FN int operator()(int i) const { return kX16rSimdFin64[i]; }
};

// qb: the lane's NTT buffer (the kernel's LDS, lanes interleaved qs apart; a local array in single())
X16R_FN __attribute__((always_inline)) void simd512(const u8* data, int n, u8* out, int16_t* qb, int qs = 1,
                                                    const int16_t* pw = kX16rSimdPw, const int16_t* yn = kX16rSimdYn,
                                                    const int16_t* yf = kX16rSimdYf) {  // 0 < n < 128
    u32 st[32];
    for (int i = 0; i < 32; ++i) st[i] = kSimdIV[i];
    u8 buf[128];
    // the message block, then the final (length) block: one copy of the rounds over the NTT buffer
    // serves both (the loop is kept rolled); a 64-byte input's final block -- X16R steps 1..15 --
    // takes the constant expansion instead of a second NTT
#pragma unroll 1
    for (int b = 0; b < 2; ++b) {
        zero(buf, 128);
        if (b == 0) {
            cpy(buf, data, n);
        } else {
            st64(buf, u64(n) * 8);
            if (n == 64) {
                simd_rounds(st, buf, SimdQFin64{});
                break;
            }
        }
        simd_expand(buf, b == 1, qb, qs, pw, yn, yf, b == 0 && n == 64);
        simd_rounds(st, buf, SimdQBuf{qb, qs});
    }
    for (int i = 0; i < 16; ++i) st32(out + 4 * i, st[i]);
}

// ================================================================ ECHO-512 (slot 10)
X16R_FN void echo_compress(u32 v[8][4], const u8 m[128], u64 counter_bits, const u32* T) {
    u32 w[16][4];
    for (int i = 0; i < 8; ++i)
        for (int c = 0; c < 4; ++c) {
            w[i][c] = v[i][c];
            w[8 + i][c] = ld32(m + 16 * i + 4 * c);
        }
    u64 k = counter_bits;
    for (int r = 0; r < 10; ++r) {
        for (int i = 0; i < 16; ++i) {
            aes_round_w(w[i], u32(k), u32(k >> 32), T);
            ++k;
            aes_round_w(w[i], 0, 0, T);
        }
        u32 t[16][4];
        for (int j = 0; j < 4; ++j)
            for (int i = 0; i < 4; ++i)
                for (int c = 0; c < 4; ++c) t[4 * j + i][c] = w[4 * ((j + i) & 3) + i][c];
        for (int j = 0; j < 4; ++j)
            for (int c = 0; c < 4; ++c) {
                const u32 a0 = t[4 * j][c], a1 = t[4 * j + 1][c], a2 = t[4 * j + 2][c], a3 = t[4 * j + 3][c];
                const u32 x0 = xtime4(a0), x1 = xtime4(a1), x2 = xtime4(a2), x3 = xtime4(a3);
                w[4 * j + 0][c] = x0 ^ x1 ^ a1 ^ a2 ^ a3;
                w[4 * j + 1][c] = a0 ^ x1 ^ x2 ^ a2 ^ a3;
                w[4 * j + 2][c] = a0 ^ a1 ^ x2 ^ x3 ^ a3;
                w[4 * j + 3][c] = x0 ^ a0 ^ a1 ^ a2 ^ x3;
            }
    }
    for (int i = 0; i < 8; ++i)
        for (int c = 0; c < 4; ++c) v[i][c] ^= ld32(m + 16 * i + 4 * c) ^ w[i][c] ^ w[8 + i][c];
}

X16R_FN void echo512(const u8* data, int n, u8* out, const u32* T = kX16rAesT) {  // 0 < n < 110
    u32 v[8][4];
    for (int i = 0; i < 8; ++i) {
        v[i][0] = 0x0200;  // 512, 128-bit little-endian
        v[i][1] = v[i][2] = v[i][3] = 0;
    }
    const u64 bits = u64(n) * 8;
    u8 buf[128];
    zero(buf, 128);
    cpy(buf, data, n);
    buf[n] = 0x80;
    buf[110] = 0x00;
    buf[111] = 0x02;
    st64(buf + 112, bits);
    echo_compress(v, buf, bits, T);
    for (int i = 0; i < 4; ++i)
        for (int c = 0; c < 4; ++c) st32(out + 16 * i + 4 * c, v[i][c]);
}

// ================================================================ Hamsi-512 (slot 11)
constexpr int kHamsiSlot[32] = {0, 1, 16, 17, 2, 3, 18, 19, 20, 21, 4, 5, 22, 23, 6, 7,
                                8, 9, 24, 25, 10, 11, 26, 27, 28, 29, 12, 13, 30, 31, 14, 15};

X16R_FN void hamsi_sbox(u32& a, u32& b, u32& c, u32& d) {
    u32 t = a;
    a &= c; a ^= d; c ^= b; c ^= a; d |= t; d ^= b; t ^= c; b = d; d |= t; d ^= a;
    a &= b; t ^= a; b ^= d; b ^= t; a = c; c = b; b = d; d = ~t;
}
X16R_FN void hamsi_L(u32& a, u32& b, u32& c, u32& d) {
    a = rl32(a, 13);
    c = rl32(c, 3);
    b ^= a ^ c;
    d ^= c ^ (a << 3);
    b = rl32(b, 1);
    d = rl32(d, 7);
    a ^= b ^ d;
    c ^= d ^ (b << 7);
    a = rl32(a, 5);
    c = rl32(c, 22);
}

X16R_FN void hamsi_block(u32 h[16], const u8 blk[8], bool fin) {
    u32 m[16];
    for (int w = 0; w < 16; ++w) m[w] = 0;
    for (int u = 0; u < 8; ++u)
        for (int v = 0; v < 8; ++v)
            if ((blk[u] >> v) & 1)
                for (int w = 0; w < 16; ++w) m[w] ^= kX16rHamsiT[16 * (8 * u + v) + w];
    u32 mc[32];
    for (int i = 0; i < 16; ++i) { mc[i] = m[i]; mc[16 + i] = h[i]; }
    u32 s[32];
    for (int i = 0; i < 32; ++i) s[i] = mc[kHamsiSlot[i]];
    const u32* alpha = fin ? kX16rHamsiAf : kX16rHamsiAn;
    const int rounds = fin ? 12 : 6;
    for (int r = 0; r < rounds; ++r) {
        for (int i = 0; i < 32; ++i) s[i] ^= alpha[i];
        s[1] ^= u32(r);
        for (int i = 0; i < 8; ++i) hamsi_sbox(s[i], s[i + 8], s[i + 16], s[i + 24]);
        for (int i = 0; i < 8; ++i) hamsi_L(s[i], s[8 + ((i + 1) & 7)], s[16 + ((i + 2) & 7)], s[24 + ((i + 3) & 7)]);
        hamsi_L(s[0x00], s[0x02], s[0x05], s[0x07]);
        hamsi_L(s[0x10], s[0x13], s[0x15], s[0x16]);
        hamsi_L(s[0x09], s[0x0B], s[0x0C], s[0x0E]);
        hamsi_L(s[0x19], s[0x1A], s[0x1C], s[0x1F]);
    }
    for (int i = 0; i < 8; ++i) {
        h[i] ^= s[i];
        h[8 + i] ^= s[16 + i];
    }
}

X16R_FN void hamsi512(const u8* data, int n, u8* out) {
    u32 h[16];
    for (int i = 0; i < 16; ++i) h[i] = kX16rHamsiIv[i];
    const u64 bits = u64(n) * 8;
    for (; n >= 8; n -= 8, data += 8) hamsi_block(h, data, false);
    u8 last[8], len[8];
    zero(last, 8);
    cpy(last, data, n);
    last[n] = 0x80;
    hamsi_block(h, last, false);
    stb64(len, bits);
    hamsi_block(h, len, true);
    for (int i = 0; i < 16; ++i) stb32(out + 4 * i, h[i]);
}

// ================================================================ Fugue-512 (slot 12)
X16R_FN void fugue_smix(u32& x0, u32& x1, u32& x2, u32& x3, const u32* mt) {
    const u32 x[4] = {x0, x1, x2, x3};
    u32 c[4] = {0, 0, 0, 0}, r[4] = {0, 0, 0, 0};
    for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 4; ++k) {
            const u32 t = mt[256 * k + ((x[j] >> (24 - 8 * k)) & 0xFF)];
            c[j] ^= t;
            if (k != j) r[k] ^= t;
        }
    x0 = ((c[0] ^ r[0]) & 0xFF000000u) | ((c[1] ^ r[1]) & 0x00FF0000u) | ((c[2] ^ r[2]) & 0x0000FF00u) |
         ((c[3] ^ r[3]) & 0x000000FFu);
    x1 = ((c[1] ^ (r[0] << 8)) & 0xFF000000u) | ((c[2] ^ (r[1] << 8)) & 0x00FF0000u) |
         ((c[3] ^ (r[2] << 8)) & 0x0000FF00u) | ((c[0] ^ (r[3] >> 24)) & 0x000000FFu);
    x2 = ((c[2] ^ (r[0] << 16)) & 0xFF000000u) | ((c[3] ^ (r[1] << 16)) & 0x00FF0000u) |
         ((c[0] ^ (r[2] >> 16)) & 0x0000FF00u) | ((c[1] ^ (r[3] >> 16)) & 0x000000FFu);
    x3 = ((c[3] ^ (r[0] << 24)) & 0xFF000000u) | ((c[0] ^ (r[1] >> 8)) & 0x00FF0000u) |
         ((c[1] ^ (r[2] >> 8)) & 0x0000FF00u) | ((c[2] ^ (r[3] >> 8)) & 0x000000FFu);
}
// Physical rotations (the host keeps the columns as a ring with a moving offset; on the GPU a
// runtime offset turns every column access into a scratch-memory access, while the unrolled
// rotations stay in registers: 41 vs 271 us per 16k-header launch, profiles/README r5k).
X16R_FN void fugue_ror(u32 S[36], int n) {
    u32 t[36];
    for (int i = 0; i < 36; ++i) t[(i + n) % 36] = S[i];
    for (int i = 0; i < 36; ++i) S[i] = t[i];
}
X16R_FN void fugue_cmix_sub(u32 S[36], const u32* mt) {
    fugue_ror(S, 3);
    S[0] ^= S[4]; S[1] ^= S[5]; S[2] ^= S[6];
    S[18] ^= S[4]; S[19] ^= S[5]; S[20] ^= S[6];
    fugue_smix(S[0], S[1], S[2], S[3], mt);
}
X16R_FN void fugue_word(u32 S[36], u32 I, const u32* mt) {
    S[22] ^= S[0];
    S[0] = I;
    S[8] ^= S[0];
    S[1] ^= S[24];
    S[4] ^= S[27];
    S[7] ^= S[30];
    for (int k = 0; k < 4; ++k) fugue_cmix_sub(S, mt);
}
constexpr u32 kFugueIV[16] = {0x8807a57e, 0xe616af75, 0xc5d3e4db, 0xac9ab027, 0xd915f117, 0xb6eecc54,
                              0x06e8020b, 0x4a92efd1, 0xaac6e2c9, 0xddb21398, 0xcae65838, 0x437f203f,
                              0x25ea78e7, 0x951fddd6, 0xda6ed11d, 0xe13e3567};
constexpr int kFugueG[4][4] = {{4, 9, 18, 27}, {4, 10, 18, 27}, {4, 10, 19, 27}, {4, 10, 19, 28}};
constexpr int kFugueOut[16] = {1, 2, 3, 4, 9, 10, 11, 12, 18, 19, 20, 21, 27, 28, 29, 30};

X16R_FN void fugue512(const u8* data, int n, u8* out, const u32* mt = kX16rFugueMt) {
    u32 S[36];
    for (int i = 0; i < 36; ++i) S[i] = 0;
    for (int i = 0; i < 16; ++i) S[20 + i] = kFugueIV[i];
    const u64 bits = u64(n) * 8;
    for (; n >= 4; n -= 4, data += 4) fugue_word(S, ldb32(data), mt);
    if (n) {
        u8 w[4] = {0, 0, 0, 0};
        cpy(w, data, n);
        fugue_word(S, ldb32(w), mt);
    }
    fugue_word(S, u32(bits >> 32), mt);
    fugue_word(S, u32(bits), mt);
    for (int i = 0; i < 32; ++i) fugue_cmix_sub(S, mt);
    for (int i = 0; i < 13; ++i)
        for (int k = 0; k < 4; ++k) {
            for (int j = 0; j < 4; ++j) S[kFugueG[k][j]] ^= S[0];
            fugue_ror(S, k == 3 ? 8 : 9);
            fugue_smix(S[0], S[1], S[2], S[3], mt);
        }
    for (int j = 0; j < 4; ++j) S[kFugueG[0][j]] ^= S[0];
    for (int i = 0; i < 16; ++i) stb32(out + 4 * i, S[kFugueOut[i]]);
}

// ================================================================ Shabal-512 (slot 13)
X16R_FN void shabal_perm(u32 A[12], u32 B[16], const u32 C[16], const u32 M[16]) {
    for (int i = 0; i < 16; ++i) B[i] = rl32(B[i], 17);
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 16; ++i) {
            const int a = (i + 16 * j) % 12, ap = (i + 16 * j + 11) % 12;
            const u32 v = A[a] ^ (rl32(A[ap], 15) * 5u) ^ C[(8 - i + 16) % 16];
            A[a] = (v * 3u) ^ B[(i + 13) % 16] ^ (B[(i + 9) % 16] & ~B[(i + 6) % 16]) ^ M[i];
            B[i] = ~(rl32(B[i], 1) ^ A[a]);
        }
    for (int j = 0; j < 36; ++j) A[j % 12] += C[(j + 3) % 16];
}

X16R_FN void shabal512(const u8* data, int n, u8* out) {
    u32 A[12], B[16], C[16], M[16];
    for (int i = 0; i < 12; ++i) A[i] = kX16rShabalA[i];
    for (int i = 0; i < 16; ++i) { B[i] = kX16rShabalB[i]; C[i] = kX16rShabalC[i]; }
    u64 W = 1;
    for (; n >= 64; n -= 64, data += 64) {
        for (int i = 0; i < 16; ++i) M[i] = ld32(data + 4 * i);
        for (int i = 0; i < 16; ++i) B[i] += M[i];
        A[0] ^= u32(W);
        A[1] ^= u32(W >> 32);
        shabal_perm(A, B, C, M);
        for (int i = 0; i < 16; ++i) C[i] -= M[i];
        for (int i = 0; i < 16; ++i) swp(B[i], C[i]);
        ++W;
    }
    u8 last[64];
    zero(last, 64);
    cpy(last, data, n);
    last[n] = 0x80;
    for (int i = 0; i < 16; ++i) M[i] = ld32(last + 4 * i);
    for (int i = 0; i < 16; ++i) B[i] += M[i];
    for (int k = 0; k < 4; ++k) {
        if (k)
            for (int i = 0; i < 16; ++i) swp(B[i], C[i]);
        A[0] ^= u32(W);
        A[1] ^= u32(W >> 32);
        shabal_perm(A, B, C, M);
    }
    for (int i = 0; i < 16; ++i) st32(out + 4 * i, B[i]);
}

// ================================================================ Whirlpool (slot 14)
X16R_FN void whirl_round(const u64 a[8], const u64 k[8], u64 out[8], const u64* T) {
    for (int i = 0; i < 8; ++i) {
        u64 v = k[i];
        for (int j = 0; j < 8; ++j) v ^= T[256 * j + u8(a[(i - j) & 7] >> (8 * j))];
        out[i] = v;
    }
}

X16R_FN void whirl_compress(u64 H[8], const u8 blk[64], const u64* T) {
    u64 K[8], st[8], m[8], tmp[8];
    for (int i = 0; i < 8; ++i) {
        m[i] = ld64(blk + 8 * i);
        K[i] = H[i];
        st[i] = m[i] ^ K[i];
    }
    for (int r = 1; r <= 10; ++r) {
        const u64 c[8] = {kX16rWhirlRc[r], 0, 0, 0, 0, 0, 0, 0};
        whirl_round(K, c, tmp, T);
        for (int i = 0; i < 8; ++i) K[i] = tmp[i];
        whirl_round(st, K, tmp, T);
        for (int i = 0; i < 8; ++i) st[i] = tmp[i];
    }
    for (int i = 0; i < 8; ++i) H[i] ^= st[i] ^ m[i];
}

X16R_FN void whirlpool512(const u8* data, int n, u8* out, const u64* T = kX16rWhirlT) {
    u64 H[8];
    for (int i = 0; i < 8; ++i) H[i] = 0;
    const u64 bits = u64(n) * 8;
    for (; n >= 64; n -= 64, data += 64) whirl_compress(H, data, T);
    u8 buf[128];
    zero(buf, 128);
    cpy(buf, data, n);
    buf[n] = 0x80;
    const int len = n < 32 ? 64 : 128;
    stb64(buf + len - 8, bits);
    whirl_compress(H, buf, T);
    if (len == 128) whirl_compress(H, buf + 64, T);
    for (int i = 0; i < 8; ++i) st64(out + 8 * i, H[i]);
}

// ================================================================ SHA-512 (slot 15)
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

X16R_FN void sha512_compress(u64 s[8], const u8* block) {
    u64 w[80];
    for (int i = 0; i < 16; ++i) w[i] = ldb64(block + 8 * i);
    for (int i = 16; i < 80; ++i) {
        const u64 a = w[i - 15], b = w[i - 2];
        w[i] = w[i - 16] + (rr64(a, 1) ^ rr64(a, 8) ^ (a >> 7)) + w[i - 7] + (rr64(b, 19) ^ rr64(b, 61) ^ (b >> 6));
    }
    u64 A = s[0], B = s[1], C = s[2], D = s[3], E = s[4], F = s[5], G = s[6], H = s[7];
    for (int i = 0; i < 80; ++i) {
        const u64 t1 = H + (rr64(E, 14) ^ rr64(E, 18) ^ rr64(E, 41)) + ((E & F) ^ (~E & G)) + kSha512K[i] + w[i];
        const u64 t2 = (rr64(A, 28) ^ rr64(A, 34) ^ rr64(A, 39)) + ((A & B) ^ (A & C) ^ (B & C));
        H = G; G = F; F = E; E = D + t1; D = C; C = B; B = A; A = t1 + t2;
    }
    s[0] += A; s[1] += B; s[2] += C; s[3] += D; s[4] += E; s[5] += F; s[6] += G; s[7] += H;
}

X16R_FN void sha512(const u8* data, int n, u8* out) {  // n < 112: one padded block
    u64 s[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    u8 buf[128];
    zero(buf, 128);
    cpy(buf, data, n);
    buf[n] = 0x80;
    stb64(buf + 120, u64(n) * 8);
    sha512_compress(s, buf);
    for (int i = 0; i < 8; ++i) stb64(out + 8 * i, s[i]);
}

// ================================================================ Tiger-192, zero-padded (X16RV2)
X16R_FN void tiger_rnd(u64& A, u64& B, u64& C, u64 xv, u64 mul, const u64* T) {
    C ^= xv;
    A -= T[u8(C)] ^ T[256 + u8(C >> 16)] ^ T[512 + u8(C >> 32)] ^ T[768 + u8(C >> 48)];
    B += T[768 + u8(C >> 8)] ^ T[512 + u8(C >> 24)] ^ T[256 + u8(C >> 40)] ^ T[u8(C >> 56)];
    B *= mul;
}
X16R_FN void tiger_pass(u64& A, u64& B, u64& C, const u64 x[8], u64 mul, const u64* T) {
    tiger_rnd(A, B, C, x[0], mul, T); tiger_rnd(B, C, A, x[1], mul, T); tiger_rnd(C, A, B, x[2], mul, T);
    tiger_rnd(A, B, C, x[3], mul, T); tiger_rnd(B, C, A, x[4], mul, T); tiger_rnd(C, A, B, x[5], mul, T);
    tiger_rnd(A, B, C, x[6], mul, T); tiger_rnd(B, C, A, x[7], mul, T);
}
X16R_FN void tiger_schedule(u64 x[8]) {
    x[0] -= x[7] ^ 0xA5A5A5A5A5A5A5A5ULL; x[1] ^= x[0]; x[2] += x[1]; x[3] -= x[2] ^ ((~x[1]) << 19);
    x[4] ^= x[3]; x[5] += x[4]; x[6] -= x[5] ^ ((~x[4]) >> 23); x[7] ^= x[6];
    x[0] += x[7]; x[1] -= x[0] ^ ((~x[7]) << 19); x[2] ^= x[1]; x[3] += x[2];
    x[4] -= x[3] ^ ((~x[2]) >> 23); x[5] ^= x[4]; x[6] += x[5]; x[7] -= x[6] ^ 0x0123456789ABCDEFULL;
}
X16R_FN void tiger_compress(const u64 xin[8], u64 st[3], const u64* T) {
    u64 a = st[0], b = st[1], c = st[2], x[8];
    for (int i = 0; i < 8; ++i) x[i] = xin[i];
    tiger_pass(a, b, c, x, 5, T);
    tiger_schedule(x);
    tiger_pass(c, a, b, x, 7, T);
    tiger_schedule(x);
    tiger_pass(b, c, a, x, 9, T);
    st[0] = a ^ st[0];
    st[1] = b - st[1];
    st[2] = c + st[2];
}

X16R_FN void tiger192_padded(const u8* data, int n, u8* out, const u64* T = kX16rTiger) {
    u64 st[3] = {0x0123456789ABCDEFULL, 0xFEDCBA9876543210ULL, 0xF096A5B4C3B2E187ULL};
    u64 x[8];
    const u64 bits = u64(n) * 8;
    for (; n >= 64; n -= 64, data += 64) {
        for (int i = 0; i < 8; ++i) x[i] = ld64(data + 8 * i);
        tiger_compress(x, st, T);
    }
    u8 buf[128];
    zero(buf, 128);
    cpy(buf, data, n);
    buf[n] = 0x01;
    const int len = n < 56 ? 64 : 128;
    st64(buf + len - 8, bits);
    for (int off = 0; off < len; off += 64) {
        for (int i = 0; i < 8; ++i) x[i] = ld64(buf + off + 8 * i);
        tiger_compress(x, st, T);
    }
    zero(out, 64);
    for (int i = 0; i < 3; ++i) st64(out + 8 * i, st[i]);
}

// ================================================================ dispatch
// Slot `algo` (0..15) of the chain, or 16 = Tiger-192 (zero-padded to 64 bytes).
X16R_FN void single(int algo, const u8* in, int n, u8* out) {
    switch (algo) {
        case 0: blake512(in, n, out); break;
        case 1: bmw512(in, n, out); break;
        case 2: groestl512(in, n, out); break;
        case 3: jh512(in, n, out); break;
        case 4: keccak512(in, n, out); break;
        case 5: skein512(in, n, out); break;
        case 6: luffa512(in, n, out); break;
        case 7: cubehash512(in, n, out); break;
        case 8: shavite512(in, n, out); break;
        case 9: {
            int16_t q[256];
            simd512(in, n, out, q);
            break;
        }
        case 10: echo512(in, n, out); break;
        case 11: hamsi512(in, n, out); break;
        case 12: fugue512(in, n, out); break;
        case 13: shabal512(in, n, out); break;
        case 14: whirlpool512(in, n, out); break;
        case 15: sha512(in, n, out); break;
        default: tiger192_padded(in, n, out); break;
    }
}

// GetHashSelection (src/hash.h:320-327): nibble 48 + i of hashPrevBlock (storage bytes).
X16R_FN int selection(const u8 prev_le[32], int index) {
    const int i = 63 - (48 + index);
    return (i % 2 == 1) ? (prev_le[i / 2] >> 4) : (prev_le[i / 2] & 0x0F);
}

// One chain step: slot `algo` over `in` (n bytes), X16RV2's Tiger pre-hash for slots 4, 6, 15.
X16R_FN void step(int algo, bool v2, const u8* in, int n, u8* out) {
    if (v2 && (algo == 4 || algo == 6 || algo == 15)) {
        u8 t[64];
        tiger192_padded(in, n, t);
        single(algo, t, 64, out);
    } else {
        single(algo, in, n, out);
    }
}

}  // namespace x16rd
