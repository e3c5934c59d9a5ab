// Equihash(200,9) device helpers shared by the two gfx950 solvers (equihash.hip: global
// slot atomics; equihash_ps.hip: private per-workgroup slot segments) and the batch verifier.
// Row convention: words w[1..7] hold the 224-bit big-endian leaf/row string, digit d_j = bits
// [20j, 20j+20); word 0 is free for the row's back-pointer. CPU golden model:
// csrc/pow/equihash.cpp (the reference has no Equihash: SURVEY §0.4 / Appendix D).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_params.h"

#ifndef NX_DEV
#define NX_DEV __device__ __forceinline__
#endif

#define EQ_MAX_CHAIN 64  // rows walked per chain of equal 8-bit sub-digits (longer chains are dropped);
                         // 24 cut chains in ~0.03 % of nonces (profiles r3zb), each a host re-solve

// digit j (20 bits) of a row held as words w[1..7] (w[1] = bits 0..31).
template <int J>
NX_DEV uint32_t eq_digit(const uint32_t* w) {
    constexpr int off = 20 * J;
    constexpr int q = off / 32 + 1;
    constexpr int o = off % 32;
    if constexpr (o + 20 <= 32) {
        return (w[q] >> (32 - o - 20)) & 0xFFFFFu;
    } else {
        return ((w[q] << (o + 20 - 32)) | (w[q + 1] >> (64 - o - 20))) & 0xFFFFFu;
    }
}

// true if bits [20*J, 200) of the row are all zero
template <int J>
NX_DEV bool eq_zero_from(const uint32_t* w) {
    constexpr int off = 20 * J;
    constexpr int q = off / 32 + 1;
    constexpr int o = off % 32;
    uint32_t acc = o ? (w[q] & (0xFFFFFFFFu >> o)) : w[q];
#pragma unroll
    for (int i = q + 1; i <= 7; ++i) acc |= w[i];
    return acc == 0;
}

// ------------------------------------------------------------------ BLAKE2b
__constant__ static const uint8_t eq_sigma[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

// 64-bit rotate as two v_alignbit_b32 on the halves (the generic lowering is four
// shifts + two ORs); N is a literal at every call site.
template <int N>
NX_DEV uint64_t eq_rotr(uint64_t x) {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if constexpr (N == 32) {
        return ((uint64_t)lo << 32) | hi;
    } else if constexpr (N < 32) {
        return ((uint64_t)__builtin_amdgcn_alignbit(lo, hi, N) << 32) | __builtin_amdgcn_alignbit(hi, lo, N);
    } else {
        return ((uint64_t)__builtin_amdgcn_alignbit(hi, lo, N - 32) << 32) | __builtin_amdgcn_alignbit(lo, hi, N - 32);
    }
}

#define EQ_G(a, b, c, d, x, y)                       \
    do {                                             \
        v[a] = v[a] + v[b] + (x); v[d] = eq_rotr<32>(v[d] ^ v[a]); \
        v[c] = v[c] + v[d];       v[b] = eq_rotr<24>(v[b] ^ v[c]); \
        v[a] = v[a] + v[b] + (y); v[d] = eq_rotr<16>(v[d] ^ v[a]); \
        v[c] = v[c] + v[d];       v[b] = eq_rotr<63>(v[b] ^ v[c]); \
    } while (0)

NX_DEV void eq_blake2b_final(const uint64_t h0[8], const uint64_t m[16], uint64_t t0, uint64_t out[8]) {
    const uint64_t iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                            0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    uint64_t v[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) { v[i] = h0[i]; v[i + 8] = iv[i]; }
    v[12] ^= t0;
    v[14] = ~v[14];
#pragma unroll
    for (int r = 0; r < 12; ++r) {
        EQ_G(0, 4, 8, 12, m[eq_sigma[r][0]], m[eq_sigma[r][1]]);
        EQ_G(1, 5, 9, 13, m[eq_sigma[r][2]], m[eq_sigma[r][3]]);
        EQ_G(2, 6, 10, 14, m[eq_sigma[r][4]], m[eq_sigma[r][5]]);
        EQ_G(3, 7, 11, 15, m[eq_sigma[r][6]], m[eq_sigma[r][7]]);
        EQ_G(0, 5, 10, 15, m[eq_sigma[r][8]], m[eq_sigma[r][9]]);
        EQ_G(1, 6, 11, 12, m[eq_sigma[r][10]], m[eq_sigma[r][11]]);
        EQ_G(2, 7, 8, 13, m[eq_sigma[r][12]], m[eq_sigma[r][13]]);
        EQ_G(3, 4, 9, 14, m[eq_sigma[r][14]], m[eq_sigma[r][15]]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = h0[i] ^ v[i] ^ v[i + 8];
}

// The 25-byte leaf `half` (0/1) of a 50-byte BLAKE2b digest as big-endian words w[1..7] (w[0] = 0).
NX_DEV void eq_leaf_words(const uint64_t out[8], int half, uint32_t w[8]) {
    w[0] = 0;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int pos = half * 25 + 4 * i + k;
            const uint32_t byte = (4 * i + k < 25) ? (uint32_t)((out[pos >> 3] >> (8 * (pos & 7))) & 0xFF) : 0u;
            v = (v << 8) | byte;
        }
        w[i + 1] = v;
    }
}

// BLAKE2b of the instance's message words with le32(g) appended at byte `input_len`
// (one compression: input_len + 4 <= 128).
NX_DEV void eq_digest(const uint64_t* msg16, const uint64_t h0[8], uint32_t input_len, uint32_t g, uint64_t out[8]) {
    uint64_t m[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = msg16[i];
    const uint32_t wi = input_len >> 3, sh = (input_len & 7) * 8;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if ((uint32_t)i == wi) m[i] |= (uint64_t)g << sh;
        if (sh > 32 && (uint32_t)i == wi + 1) m[i] |= (uint64_t)g >> (64 - sh);
    }
    eq_blake2b_final(h0, m, (uint64_t)input_len + 4, out);
}

// First word (of w[1..7]) that still carries bits at level L: bits [20L, 200).
// From level 5 on that is word >= 4, so only the second 16-byte half of a
// 32-byte row slot is read or written (levels 5..8: half the row traffic).
constexpr int eq_first_word(int level) { return (20 * level) / 32 + 1; }
#ifdef EQ_NO_HALF
constexpr bool eq_half_row(int) { return false; }
#else
constexpr bool eq_half_row(int level) { return eq_first_word(level) >= 4; }
#endif

// XOR of two staged rows of level L-1 into the level-L row x (words of
// levels < first meaningful word are zero / never read).
template <int L>
NX_DEV void eq_xor_rows(const uint32_t* a, const uint32_t* b, uint32_t x[8]) {
    constexpr int k0 = eq_half_row(L - 1) ? 4 : 1;
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = (k >= k0) ? (a[k] ^ b[k]) : 0u;
}


// From level 5 on (eq_half_row) bits [0, 20L) of a row are zero and bits [20L, 20L + 12) are
// its bucket, so the row is its back-pointer plus bits 112..207 (words 4..7 shifted by 16): one
// 16-byte store and load instead of two. Level 5 is the only level whose word 4 has non-zero
// bits above bit 112 (its bucket, bits 100..111), restored from the bucket on unpacking.
NX_DEV uint4 eq_pack16(uint32_t ref, const uint32_t x[8]) {
    return make_uint4(ref, (x[4] << 16) | (x[5] >> 16), (x[5] << 16) | (x[6] >> 16), (x[6] << 16) | (x[7] >> 16));
}
// Words 4..7 of a packed row; `hi` = the known top half of word 4 (bucket << 16 at level 5, else 0).
NX_DEV void eq_unpack16(uint4 v, uint32_t hi, uint32_t w[8]) {
    w[4] = hi | (v.y >> 16);
    w[5] = (v.y << 16) | (v.z >> 16);
    w[6] = (v.z << 16) | (v.w >> 16);
    w[7] = v.w << 16;
}

// Reconstruct the 512 leaf indices of every candidate, reject duplicate trees
// early (most final-round collisions reuse a row: they are caught while the
// tree is still <= 64 wide), canonicalise the order, and append valid
// solutions. EQ_RECON_GROUPS workgroups per instance stride over candidates.
// `refs` is one instance's [LEVELS][BUCKETS][STRIDE] back-pointer table: a node id s =
// bucket * STRIDE + index, and a level > 0 entry is (parent bucket << 20 | index a << 10 | index b)
// into the level below (STRIDE <= 1024). `c` = (count, then node pairs) of level-8 candidates,
// `sb` = (count, then 512-index solutions). One workgroup of BLOCK threads per candidate,
// grid-strided over them.
template <uint32_t STRIDE, int BLOCK>
NX_DEV void eq_reconstruct_body(const uint32_t* refs, const uint32_t* c, uint32_t* sb) {
    __shared__ uint32_t cur[512];
    __shared__ uint32_t tmp[512];
    __shared__ int bad;
    __shared__ uint32_t slot;
    const uint32_t ncand = min(c[0], (uint32_t)EQ_MAX_CAND);
    for (uint32_t cand = blockIdx.x; cand < ncand; cand += gridDim.x) {
        __syncthreads();  // previous iteration done with the LDS arrays
        if (threadIdx.x == 0) {
            cur[0] = c[1 + 2 * cand];
            cur[1] = c[2 + 2 * cand];
            bad = 0;
        }
        __syncthreads();
        uint32_t width = 2;
        for (int level = 8; level >= 1; --level) {
            for (uint32_t t = threadIdx.x; t < width; t += BLOCK) {
                const uint32_t s = cur[t];
                const uint32_t ref = refs[((size_t)level * EQ_BUCKETS) * STRIDE + s];
                const uint32_t pb = ref >> 20;
                tmp[2 * t] = pb * STRIDE + ((ref >> 10) & 1023u);
                tmp[2 * t + 1] = pb * STRIDE + (ref & 1023u);
            }
            __syncthreads();
            width *= 2;
            for (uint32_t t = threadIdx.x; t < width; t += BLOCK) cur[t] = tmp[t];
            __syncthreads();
            if (width <= 64) {  // a repeated row at any level means repeated leaves
                const uint32_t npairs = width * (width - 1) / 2;
                for (uint32_t q = threadIdx.x; q < npairs; q += BLOCK) {
                    uint32_t a = 0, rem = q;
                    while (rem >= width - 1 - a) { rem -= width - 1 - a; ++a; }
                    if (cur[a] == cur[a + 1 + rem]) bad = 1;
                }
                __syncthreads();
                if (bad) break;
            }
        }
        if (bad) continue;
        for (uint32_t t = threadIdx.x; t < 512; t += BLOCK) {
            const uint32_t s = cur[t];
            cur[t] = refs[s];
        }
        __syncthreads();
        // canonical order: every node's left subtree starts with the smaller index
        for (uint32_t sz = 1; sz < 512; sz *= 2) {
            for (uint32_t node = threadIdx.x; node < 512 / (2 * sz); node += BLOCK) {
                const uint32_t l = node * 2 * sz, r = l + sz;
                if (cur[l] > cur[r]) {
                    for (uint32_t k = 0; k < sz; ++k) {
                        const uint32_t x = cur[l + k];
                        cur[l + k] = cur[r + k];
                        cur[r + k] = x;
                    }
                }
            }
            __syncthreads();
        }
        // full duplicate check on a bitonic-sorted copy
        for (uint32_t t = threadIdx.x; t < 512; t += BLOCK) tmp[t] = cur[t];
        __syncthreads();
        for (uint32_t k = 2; k <= 512; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t t = threadIdx.x; t < 512; t += BLOCK) {
                    const uint32_t ixj = t ^ j;
                    if (ixj > t) {
                        const bool up = (t & k) == 0;
                        const uint32_t a = tmp[t], b = tmp[ixj];
                        if ((a > b) == up) {
                            tmp[t] = b;
                            tmp[ixj] = a;
                        }
                    }
                }
                __syncthreads();
            }
        }
        for (uint32_t t = threadIdx.x; t < 511; t += BLOCK)
            if (tmp[t] == tmp[t + 1]) bad = 1;
        __syncthreads();
        if (bad) continue;
        if (threadIdx.x == 0) slot = atomicAdd(&sb[0], 1u);
        __syncthreads();
        if (slot < EQ_MAX_SOL)
            for (uint32_t t = threadIdx.x; t < 512; t += BLOCK) sb[1 + slot * 512 + t] = cur[t];
    }
}

// Leaf indices of every candidate of a pair-log solver (equihash_cb.hip): node ids at level L are
// row ids, children(L, id, a, b) gives the two level-(L-1) ids a row was made of, and level-0 ids
// are leaf indices. Same pruning, canonical order and duplicate check as eq_reconstruct_body.
template <int BLOCK, class Children>
NX_DEV void eq_reconstruct_tree(Children children, const uint32_t* c, uint32_t* sb) {
    __shared__ uint32_t cur[512];
    __shared__ uint32_t tmp[512];
    __shared__ int bad;
    __shared__ uint32_t slot;
    const uint32_t ncand = min(c[0], (uint32_t)EQ_MAX_CAND);
    for (uint32_t cand = blockIdx.x; cand < ncand; cand += gridDim.x) {
        __syncthreads();  // previous iteration done with the LDS arrays
        if (threadIdx.x == 0) {
            cur[0] = c[1 + 2 * cand];
            cur[1] = c[2 + 2 * cand];
            bad = 0;
        }
        __syncthreads();
        uint32_t width = 2;
        for (int level = 8; level >= 1; --level) {
            for (uint32_t t = threadIdx.x; t < width; t += BLOCK) {
                uint32_t a, b;
                children(level, cur[t], a, b);
                tmp[2 * t] = a;
                tmp[2 * t + 1] = b;
            }
            __syncthreads();
            width *= 2;
            for (uint32_t t = threadIdx.x; t < width; t += BLOCK) cur[t] = tmp[t];
            __syncthreads();
            if (width <= 64) {  // a repeated row at any level means repeated leaves
                const uint32_t npairs = width * (width - 1) / 2;
                for (uint32_t q = threadIdx.x; q < npairs; q += BLOCK) {
                    uint32_t a = 0, rem = q;
                    while (rem >= width - 1 - a) { rem -= width - 1 - a; ++a; }
                    if (cur[a] == cur[a + 1 + rem]) bad = 1;
                }
                __syncthreads();
                if (bad) break;
            }
        }
        if (bad) continue;
        // canonical order: every node's left subtree starts with the smaller index
        for (uint32_t sz = 1; sz < 512; sz *= 2) {
            for (uint32_t node = threadIdx.x; node < 512 / (2 * sz); node += BLOCK) {
                const uint32_t l = node * 2 * sz, r = l + sz;
                if (cur[l] > cur[r]) {
                    for (uint32_t k = 0; k < sz; ++k) {
                        const uint32_t x = cur[l + k];
                        cur[l + k] = cur[r + k];
                        cur[r + k] = x;
                    }
                }
            }
            __syncthreads();
        }
        // full duplicate check on a bitonic-sorted copy
        for (uint32_t t = threadIdx.x; t < 512; t += BLOCK) tmp[t] = cur[t];
        __syncthreads();
        for (uint32_t k = 2; k <= 512; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t t = threadIdx.x; t < 512; t += BLOCK) {
                    const uint32_t ixj = t ^ j;
                    if (ixj > t) {
                        const bool up = (t & k) == 0;
                        const uint32_t a = tmp[t], b = tmp[ixj];
                        if ((a > b) == up) {
                            tmp[t] = b;
                            tmp[ixj] = a;
                        }
                    }
                }
                __syncthreads();
            }
        }
        for (uint32_t t = threadIdx.x; t < 511; t += BLOCK)
            if (tmp[t] == tmp[t + 1]) bad = 1;
        __syncthreads();
        if (bad) continue;
        if (threadIdx.x == 0) slot = atomicAdd(&sb[0], 1u);
        __syncthreads();
        if (slot < EQ_MAX_SOL)
            for (uint32_t t = threadIdx.x; t < 512; t += BLOCK) sb[1 + slot * 512 + t] = cur[t];
    }
}
