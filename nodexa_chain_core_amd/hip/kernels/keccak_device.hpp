// Device-side Keccak permutations for gfx950.
//
// keccak_f800: 22 rounds over 25 x u32 (KawPow seed/final absorbs,
// src/crypto/ethash/lib/keccak/keccakf800.c). keccak_f1600: 24 rounds over
// 25 x u64 (ethash keccak512 for DAG items). Both are written with every lane
// index a compile-time constant so the state stays in VGPRs; 32-bit rotates
// lower to v_alignbit_b32, 64-bit rotates to a v_alignbit pair.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define NX_DEV __device__ __forceinline__

NX_DEV uint32_t nx_rotl32(uint32_t x, uint32_t n) { return __builtin_rotateleft32(x, n); }
NX_DEV uint64_t nx_rotl64(uint64_t x, uint32_t n) { return __builtin_rotateleft64(x, n); }

__constant__ static const uint64_t nx_keccak_rc[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL,
};

// One Keccak round on a 25-lane state of type T (u32 or u64); R(x, n) rotates.
#define NX_KECCAK_ROUND(T, a, R, rc)                                                           \
    do {                                                                                       \
        T c0 = a[0] ^ a[5] ^ a[10] ^ a[15] ^ a[20];                                            \
        T c1 = a[1] ^ a[6] ^ a[11] ^ a[16] ^ a[21];                                            \
        T c2 = a[2] ^ a[7] ^ a[12] ^ a[17] ^ a[22];                                            \
        T c3 = a[3] ^ a[8] ^ a[13] ^ a[18] ^ a[23];                                            \
        T c4 = a[4] ^ a[9] ^ a[14] ^ a[19] ^ a[24];                                            \
        T d0 = c4 ^ R(c1, 1), d1 = c0 ^ R(c2, 1), d2 = c1 ^ R(c3, 1), d3 = c2 ^ R(c4, 1),      \
          d4 = c3 ^ R(c0, 1);                                                                  \
        /* theta + rho + pi: b[y + 5*((2x+3y)%5)] = rot(a[x+5y] ^ d[x], rho[x+5y]) */         \
        T b0 = a[0] ^ d0;                                                                      \
        T b10 = R(a[1] ^ d1, 1);                                                               \
        T b20 = R(a[2] ^ d2, 62);                                                              \
        T b5 = R(a[3] ^ d3, 28);                                                               \
        T b15 = R(a[4] ^ d4, 27);                                                              \
        T b16 = R(a[5] ^ d0, 36);                                                              \
        T b1 = R(a[6] ^ d1, 44);                                                               \
        T b11 = R(a[7] ^ d2, 6);                                                               \
        T b21 = R(a[8] ^ d3, 55);                                                              \
        T b6 = R(a[9] ^ d4, 20);                                                               \
        T b7 = R(a[10] ^ d0, 3);                                                               \
        T b17 = R(a[11] ^ d1, 10);                                                             \
        T b2 = R(a[12] ^ d2, 43);                                                              \
        T b12 = R(a[13] ^ d3, 25);                                                             \
        T b22 = R(a[14] ^ d4, 39);                                                             \
        T b23 = R(a[15] ^ d0, 41);                                                             \
        T b8 = R(a[16] ^ d1, 45);                                                              \
        T b18 = R(a[17] ^ d2, 15);                                                             \
        T b3 = R(a[18] ^ d3, 21);                                                              \
        T b13 = R(a[19] ^ d4, 8);                                                              \
        T b14 = R(a[20] ^ d0, 18);                                                             \
        T b24 = R(a[21] ^ d1, 2);                                                              \
        T b9 = R(a[22] ^ d2, 61);                                                              \
        T b19 = R(a[23] ^ d3, 56);                                                             \
        T b4 = R(a[24] ^ d4, 14);                                                              \
        /* chi */                                                                              \
        a[0] = b0 ^ (~b1 & b2); a[1] = b1 ^ (~b2 & b3); a[2] = b2 ^ (~b3 & b4);                \
        a[3] = b3 ^ (~b4 & b0); a[4] = b4 ^ (~b0 & b1);                                        \
        a[5] = b5 ^ (~b6 & b7); a[6] = b6 ^ (~b7 & b8); a[7] = b7 ^ (~b8 & b9);                \
        a[8] = b8 ^ (~b9 & b5); a[9] = b9 ^ (~b5 & b6);                                        \
        a[10] = b10 ^ (~b11 & b12); a[11] = b11 ^ (~b12 & b13); a[12] = b12 ^ (~b13 & b14);    \
        a[13] = b13 ^ (~b14 & b10); a[14] = b14 ^ (~b10 & b11);                                \
        a[15] = b15 ^ (~b16 & b17); a[16] = b16 ^ (~b17 & b18); a[17] = b17 ^ (~b18 & b19);    \
        a[18] = b18 ^ (~b19 & b15); a[19] = b19 ^ (~b15 & b16);                                \
        a[20] = b20 ^ (~b21 & b22); a[21] = b21 ^ (~b22 & b23); a[22] = b22 ^ (~b23 & b24);    \
        a[23] = b23 ^ (~b24 & b20); a[24] = b24 ^ (~b20 & b21);                                \
        a[0] ^= (T)(rc);                                                                       \
    } while (0)

#define NX_R32(x, n) nx_rotl32((x), (n) & 31)
#define NX_R64(x, n) nx_rotl64((x), (n))

// NX_KECCAK800_ROLLED keeps the 22 rounds as a loop: ~55 live VGPRs at most, where the unrolled
// form lets the scheduler overlap rounds and, under a tight register budget (the 6-wave KawPow
// search kernel has 80), spill.
NX_DEV void keccak_f800(uint32_t a[25]) {
#ifdef NX_KECCAK800_ROLLED
#pragma unroll 1
#else
#pragma unroll
#endif
    for (int r = 0; r < 22; ++r) NX_KECCAK_ROUND(uint32_t, a, NX_R32, (uint32_t)nx_keccak_rc[r]);
}

NX_DEV void keccak_f1600(uint64_t a[25]) {
#pragma unroll 1
    for (int r = 0; r < 24; ++r) NX_KECCAK_ROUND(uint64_t, a, NX_R64, nx_keccak_rc[r]);
}

// keccak512 of exactly 64 bytes (8 u64 words) -> 8 u64 words (original Keccak padding).
NX_DEV void keccak512_64(const uint64_t in[8], uint64_t out[8]) {
    uint64_t a[25];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = in[i];
    a[8] = 0x8000000000000001ULL;
#pragma unroll
    for (int i = 9; i < 25; ++i) a[i] = 0;
    keccak_f1600(a);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = a[i];
}
