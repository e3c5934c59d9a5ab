// Equihash(200,9) batch verification on gfx950 (new; the reference has no Equihash — SURVEY §0.4 /
// Appendix D). CPU golden model: csrc/pow/equihash.cpp. The solver is equihash_ps.hip; the
// global-slot solver that lived here (one returning global atomic per row, 6.5 ms per 8 solves
// against 4.4 for the private-slot engine, profiles/README r2d-r3) was removed in round 5.
#include "equihash_device.hpp"  // BLAKE2b, digits (shared with equihash_ps.hip)

#define EQ_BLOCK 256

// ------------------------------------------------------------------ batch verify
// One 256-thread workgroup per packed solution (the extension's header check,
// models/verify.py; SURVEY K10 `eqh_verify_batch`). The 512 leaves are
// regenerated (BLAKE2b of input || le32(index / 2), half index % 2), then the
// tree is folded level by level in LDS: at level l every node's children must
// XOR to a string whose first 20*l bits are zero (all 200 at the root), the
// left subtree's first index must be smaller than the right one's, and the
// sorted index list must have no repeats — the rules of the CPU verifier
// (csrc/pow/equihash.cpp).
NX_DEV void eq_leaf(const uint64_t* msg, const uint64_t* h0, uint32_t input_len, uint32_t index, uint32_t w[8]) {
    uint64_t out[8];
    eq_digest(msg, h0, input_len, index >> 1, out);
    eq_leaf_words(out, (int)(index & 1), w);
}

// first `bits` bits of the row w[1..7] (big-endian) are zero
NX_DEV bool eq_prefix_zero(const uint32_t* w, int bits) {
    for (int i = 1; i <= 7 && bits > 0; ++i, bits -= 32) {
        const uint32_t mask = bits >= 32 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> bits);
        if (w[i] & mask) return false;
    }
    return true;
}

// The tree rules over idx[512] (already in LDS, copied to srt): leaves regenerated from the
// input, XOR-folded level by level, ordering and distinctness. Returns EQ_V_* (all threads).
struct EqVerifyLds {
    uint32_t idx[512];
    uint32_t srt[512];
    uint32_t nodes[2][512 * 8];
    uint32_t verdict;
};

NX_DEV uint32_t eq_verify_tree(const uint64_t* msg, const uint64_t* h0, uint32_t input_len, EqVerifyLds& L) {
    for (uint32_t i = threadIdx.x; i < 512; i += EQ_BLOCK) {
        uint32_t w[8];
        eq_leaf(msg, h0, input_len, L.idx[i], w);
#pragma unroll
        for (int k = 0; k < 8; ++k) L.nodes[0][i * 8 + k] = w[k];
    }
    __syncthreads();
    for (int l = 1; l <= 9; ++l) {
        const uint32_t* src = L.nodes[(l - 1) & 1];
        uint32_t* dst = L.nodes[l & 1];
        const uint32_t n = 512u >> l;
        for (uint32_t j = threadIdx.x; j < n; j += EQ_BLOCK) {
            uint32_t x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = src[(2 * j) * 8 + k] ^ src[(2 * j + 1) * 8 + k];
            if (!eq_prefix_zero(x, l == 9 ? 200 : 20 * l)) atomicMax(&L.verdict, l == 9 ? EQ_V_NONZERO : EQ_V_COLLISION);
            if (L.idx[(2 * j) << (l - 1)] >= L.idx[(2 * j + 1) << (l - 1)]) atomicMax(&L.verdict, EQ_V_ORDER);
#pragma unroll
            for (int k = 0; k < 8; ++k) dst[j * 8 + k] = x[k];
        }
        __syncthreads();
    }
    // distinct indices: bitonic sort of the copy, then adjacent compare
    for (uint32_t k = 2; k <= 512; k <<= 1) {
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            for (uint32_t t = threadIdx.x; t < 512; t += EQ_BLOCK) {
                const uint32_t o = t ^ jj;
                if (o > t) {
                    const uint32_t a = L.srt[t], b = L.srt[o];
                    if ((a > b) == ((t & k) == 0)) {
                        L.srt[t] = b;
                        L.srt[o] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t t = threadIdx.x; t < 511; t += EQ_BLOCK)
        if (L.srt[t] == L.srt[t + 1]) atomicMax(&L.verdict, EQ_V_DUPLICATE);
    __syncthreads();
    return L.verdict;
}

extern "C" __global__ __launch_bounds__(EQ_BLOCK) void eq_verify(EquihashVerifyParams p) {
    __shared__ EqVerifyLds L;
    const uint32_t s = blockIdx.x;
    if (threadIdx.x == 0) L.verdict = EQ_V_OK;
    const uint8_t* sb = (const uint8_t*)(p.sols + (size_t)s * EQ_SOL_WORDS);
    for (uint32_t i = threadIdx.x; i < 512; i += EQ_BLOCK) {
        const uint32_t bit = 21u * i, byte = bit >> 3, sh = bit & 7;
        const uint32_t v = ((uint32_t)sb[byte] << 24) | ((uint32_t)sb[byte + 1] << 16) | ((uint32_t)sb[byte + 2] << 8) |
                           (byte + 3 < 1344 ? (uint32_t)sb[byte + 3] : 0u);
        const uint32_t x = (v >> (32 - sh - 21)) & 0x1FFFFFu;
        L.idx[i] = x;
        L.srt[i] = x;
    }
    __syncthreads();
    const uint32_t v = eq_verify_tree(p.msgs + (size_t)s * 16, p.h0, p.input_len, L);
    if (threadIdx.x == 0) p.out[s] = v;
}

// The solver's own output, checked where it lies (miner/equihash devices): workgroup (k, inst)
// takes solution slot k of instance inst from the solver's [inst][1 + EQ_MAX_SOL * 512] buffer
// and applies the same rules as eq_verify, so every solution the miner counts has been checked
// independently of the rounds that produced it without a host pass over 512 BLAKE2b leaves
// (~225 us per solution on one host core). Empty slots report EQ_V_EMPTY.
extern "C" __global__ __launch_bounds__(EQ_BLOCK) void eq_verify_slots(EquihashSlotVerifyParams p) {
    __shared__ EqVerifyLds L;
    const uint32_t k = blockIdx.x, inst = blockIdx.y;
    const uint32_t* sb = p.sols + (size_t)inst * (1 + EQ_MAX_SOL * 512);
    const uint32_t n = sb[0] < EQ_MAX_SOL ? sb[0] : EQ_MAX_SOL;
    if (k >= n) {  // uniform over the workgroup
        if (threadIdx.x == 0) p.out[inst * EQ_MAX_SOL + k] = EQ_V_EMPTY;
        return;
    }
    if (threadIdx.x == 0) L.verdict = EQ_V_OK;
    for (uint32_t i = threadIdx.x; i < 512; i += EQ_BLOCK) {
        const uint32_t x = sb[1 + k * 512 + i] & 0x1FFFFFu;
        L.idx[i] = x;
        L.srt[i] = x;
    }
    __syncthreads();
    const uint32_t v = eq_verify_tree(p.msgs + (size_t)inst * 16, p.h0, p.input_len, L);
    if (threadIdx.x == 0) p.out[inst * EQ_MAX_SOL + k] = v;
}
