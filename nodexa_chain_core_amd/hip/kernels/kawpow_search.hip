// KawPow nonce search for gfx950 — per-period template.
//
// Compiled once per ProgPoW period (3 blocks) together with the header that
// csrc/pow/kawpow_codegen.cpp emits for that period (KAWPOW_PROGRAM /
// KAWPOW_DAG_MERGE with every register index and opcode baked in). Reference
// behaviour: progpow::search / hash (src/crypto/ethash/lib/ethash/progpow.cpp:
// 298-355, 553-579) — the CPU golden model lives in csrc/pow/kawpow.cpp.
//
// CDNA4 mapping
//   * one ProgPoW lane per thread; a 16-thread group is one hash; a wave64 runs
//     4 groups side by side. Each thread owns one nonce: it computes that
//     nonce's keccak-f800 seed, then its group walks the group's 16 nonces
//     (the keccak cost is paid once per nonce, not 16x).
//   * the hash is a chain of 64 dependent DAG gathers (round r+1's address
//     depends on round r's DAG merge into mix[0]), so throughput is set by how
//     many gathers are in flight per SIMD (Little's law on HBM latency), not by
//     ALU. A group therefore interleaves KP_HASHES independent hashes of its 16
//     (KP_HASHES x 32 mix VGPRs): KP_HASHES gathers are issued back to back at
//     round start and the KP_HASHES programs give the scheduler independent
//     chains to fill the latency with.
//   * the mix registers are arrays subscripted only by literals (the emitted
//     program bakes every index in), so they are scalarised into VGPRs.
//   * everything not needed inside the round loop leaves the VGPR file: the 8
//     digest words go to LDS as each hash finishes, and the keccak state words
//     2..7 are recomputed for the final absorb instead of being held live.
//   * the 16 KiB L1 (first 64 DAG items) sits in LDS; cache ops are
//     ds_read_b32 with a 12-bit masked address.
//   * each round's 256-byte DAG item is one coalesced 16 B/lane load by the
//     group (lane l takes words ((l^r)%16)*4..+3); the item index is broadcast
//     from lane r%16 with ds_bpermute (__shfl, width 16) and reduced with a
//     FastMod32 multiply-shift.
#include "kernel_params.h"
#include "keccak_device.hpp"

#ifndef KAWPOW_PROGRAM_HEADER
#define KAWPOW_PROGRAM_HEADER "kawpow_program_default.inc"
#endif
#include KAWPOW_PROGRAM_HEADER

// Tuning knobs (compile-time; ops/jit.py passes them as -D variants):
//   KP_HASHES     hashes interleaved per 16-lane group (1, 2, 4 or 8)
//   KP_MIN_WAVES  minimum waves per SIMD for __launch_bounds__ (caps VGPRs)
//   KP_NT_DAG     non-temporal DAG loads (the 4 GiB DAG has no L2 reuse)
#ifndef KP_HASHES
#define KP_HASHES 2
#endif
#if (16 % KP_HASHES) != 0
#error "KP_HASHES must divide 16"
#endif
#ifdef KP_MIN_WAVES
#define KP_BOUNDS __launch_bounds__(NODEXA_KAWPOW_BLOCK, KP_MIN_WAVES)
#else
#define KP_BOUNDS __launch_bounds__(NODEXA_KAWPOW_BLOCK)
#endif
typedef uint32_t kp_u32x4 __attribute__((ext_vector_type(4)));
NX_DEV uint4 kp_dag_load(const uint4* p) {
#ifdef KP_NT_DAG
    const kp_u32x4 v = __builtin_nontemporal_load((const kp_u32x4*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}

// x*33 for the merge ops. Left to itself the compiler folds `a*33 + b` into
// v_mad_u64_u32 (a multi-cycle integer MAD); KP_MUL33_SHIFT pins it to one
// full-rate v_lshl_add_u32 (a<<5)+a, leaving the +b as a plain add.
#ifdef KP_MUL33_SHIFT
NX_DEV uint32_t kp_mul33(uint32_t a) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 5, %1" : "=v"(r) : "v"(a));
    return r;
}
#else
NX_DEV uint32_t kp_mul33(uint32_t a) { return a * 33u; }
#endif

NX_DEV uint32_t kp_clz(uint32_t x) { return x ? (uint32_t)__builtin_clz(x) : 32u; }
NX_DEV uint32_t kp_fnv1a(uint32_t h, uint32_t d) { return (h ^ d) * 0x01000193u; }
NX_DEV uint32_t kp_fastmod(uint32_t x, const FastMod32& f) {
    const uint32_t t = __umulhi(x, f.m);
    const uint32_t q = (t + ((x - t) >> 1)) >> (f.s - 1);
    return x - q * f.d;
}

struct KpKiss {
    uint32_t z, w, jsr, jcong;
    NX_DEV uint32_t next() {
        z = 36969u * (z & 0xffffu) + (z >> 16);
        w = 18000u * (w & 0xffffu) + (w >> 16);
        jcong = 69069u * jcong + 1234567u;
        jsr ^= (jsr << 17);
        jsr ^= (jsr >> 13);
        jsr ^= (jsr << 5);
        return (((z << 16) + w) ^ jcong) + jsr;
    }
};

// "rAVENCOINKAWPOW" padding words (one byte per u32).
#define KP_PAD0 0x72u
#define KP_PAD1 0x41u
#define KP_PAD2 0x56u
#define KP_PAD3 0x45u
#define KP_PAD4 0x4Eu
#define KP_PAD5 0x43u
#define KP_PAD6 0x4Fu
#define KP_PAD7 0x49u
#define KP_PAD8 0x4Eu
#define KP_PAD9 0x4Bu
#define KP_PAD10 0x41u
#define KP_PAD11 0x57u
#define KP_PAD12 0x50u
#define KP_PAD13 0x4Fu
#define KP_PAD14 0x57u

NX_DEV void kp_seed(const uint32_t header[8], uint64_t nonce, uint32_t st2[8]) {
    uint32_t s[25];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = header[i];
    s[8] = (uint32_t)nonce;
    s[9] = (uint32_t)(nonce >> 32);
    s[10] = KP_PAD0; s[11] = KP_PAD1; s[12] = KP_PAD2; s[13] = KP_PAD3; s[14] = KP_PAD4;
    s[15] = KP_PAD5; s[16] = KP_PAD6; s[17] = KP_PAD7; s[18] = KP_PAD8; s[19] = KP_PAD9;
    s[20] = KP_PAD10; s[21] = KP_PAD11; s[22] = KP_PAD12; s[23] = KP_PAD13; s[24] = KP_PAD14;
    keccak_f800(s);
#pragma unroll
    for (int i = 0; i < 8; ++i) st2[i] = s[i];
}

NX_DEV void kp_final(const uint32_t st2[8], const uint32_t digest[8], uint32_t out[8]) {
    uint32_t s[25];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = st2[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[8 + i] = digest[i];
    s[16] = KP_PAD0; s[17] = KP_PAD1; s[18] = KP_PAD2; s[19] = KP_PAD3; s[20] = KP_PAD4;
    s[21] = KP_PAD5; s[22] = KP_PAD6; s[23] = KP_PAD7; s[24] = KP_PAD8;
    keccak_f800(s);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = s[i];
}

// The group's 16 hashes, KP_HASHES at a time. `st0/st1` are this thread's own
// nonce seed words (hash h's seed lives in lane h). Each finished hash's 8
// digest words are written to dig[h * 8 + k] (LDS, this group's 128 words).
NX_DEV void kp_group_hashes(const uint4* __restrict__ dag, const FastMod32& items, const uint32_t* l1,
                            uint32_t st0, uint32_t st1, uint32_t lane, uint32_t* dig) {
#pragma unroll 1
    for (uint32_t h0 = 0; h0 < 16; h0 += KP_HASHES) {
        uint32_t mx[KP_HASHES][32];
#pragma unroll
        for (int k = 0; k < KP_HASHES; ++k) {
            const uint32_t s0 = __shfl(st0, (int)(h0 + k), 16);
            const uint32_t s1 = __shfl(st1, (int)(h0 + k), 16);
            const uint32_t z = kp_fnv1a(0x811c9dc5u, s0);
            const uint32_t w = kp_fnv1a(z, s1);
            const uint32_t jsr = kp_fnv1a(w, lane);
            KpKiss rng{z, w, jsr, kp_fnv1a(jsr, lane)};
#pragma unroll
            for (int i = 0; i < 32; ++i) mx[k][i] = rng.next();
        }
#pragma unroll 1
        for (uint32_t r = 0; r < 64; ++r) {
            uint4 d[KP_HASHES];
            const uint32_t part = (lane ^ r) & 15;
#pragma unroll
            for (int k = 0; k < KP_HASHES; ++k) {
                const uint32_t index = kp_fastmod(__shfl(mx[k][0], (int)(r & 15), 16), items);
                d[k] = kp_dag_load(dag + (size_t)index * 16 + part);
            }
#pragma unroll
            for (int k = 0; k < KP_HASHES; ++k) KAWPOW_PROGRAM(l1, mx[k]);
#pragma unroll
            for (int k = 0; k < KP_HASHES; ++k) KAWPOW_DAG_MERGE(d[k], mx[k]);
        }
#pragma unroll
        for (int k = 0; k < KP_HASHES; ++k) {
            uint32_t lh = 0x811c9dc5u;
#pragma unroll
            for (int i = 0; i < 32; ++i) lh = kp_fnv1a(lh, mx[k][i]);
            // digest[j] = fnv1a(fnv1a(basis, lane_hash[j]), lane_hash[j + 8]); lanes 0..7 own j
            const uint32_t hi = __shfl(lh, (int)(lane + 8), 16);
            if (lane < 8) dig[(h0 + k) * 8 + lane] = kp_fnv1a(kp_fnv1a(0x811c9dc5u, lh), hi);
        }
    }
}

extern "C" __global__ KP_BOUNDS void kawpow_search(KawpowSearchParams p) {
    __shared__ uint32_t l1[4096];
    __shared__ uint32_t digs[NODEXA_KAWPOW_BLOCK * 8];
    {
        const uint4* src = (const uint4*)p.dag;
        uint4* dst = (uint4*)l1;
#pragma unroll
        for (int i = threadIdx.x; i < 1024; i += NODEXA_KAWPOW_BLOCK) dst[i] = src[i];
    }
    __syncthreads();

    const uint32_t lane = threadIdx.x & 15;
    const uint64_t nonce = p.start_nonce + (uint64_t)blockIdx.x * NODEXA_KAWPOW_BLOCK + threadIdx.x;
    uint32_t* dig = digs + (threadIdx.x & ~15u) * 8;
    {
        uint32_t st2[8];
        kp_seed(p.header, nonce, st2);
        kp_group_hashes((const uint4*)p.dag, p.items, l1, st2[0], st2[1], lane, dig);
    }
    __syncthreads();
    uint32_t st2[8], digest[8], fin[8];
    kp_seed(p.header, nonce, st2);  // recomputed: cheaper than 6 VGPRs held across the mix loop
#pragma unroll
    for (int k = 0; k < 8; ++k) digest[k] = dig[lane * 8 + k];
    kp_final(st2, digest, fin);
    const uint64_t head = ((uint64_t)__builtin_bswap32(fin[0]) << 32) | __builtin_bswap32(fin[1]);
    if (head <= p.target) {
        const uint32_t slot = atomicAdd(&p.results->count, 1u);
        if (slot < NODEXA_KAWPOW_MAX_SHARES) {
            KawpowShare* s = &p.results->shares[slot];
            s->nonce = nonce;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                s->mix[k] = digest[k];
                s->final_[k] = fin[k];
            }
        }
    }
}

// Batch hash (no target): for verification of (header, nonce, height) jobs that
// all share this period and epoch. One job per thread, grouped as in search.
extern "C" __global__ KP_BOUNDS void kawpow_hash_batch(KawpowHashParams p) {
    __shared__ uint32_t l1[4096];
    __shared__ uint32_t digs[NODEXA_KAWPOW_BLOCK * 8];
    {
        const uint4* src = (const uint4*)p.dag;
        uint4* dst = (uint4*)l1;
        for (int i = threadIdx.x; i < 1024; i += NODEXA_KAWPOW_BLOCK) dst[i] = src[i];
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 15;
    const uint32_t job = blockIdx.x * NODEXA_KAWPOW_BLOCK + threadIdx.x;
    const bool valid = job < p.num_jobs;
    const KawpowVerifyJob j = p.jobs[valid ? job : 0];
    uint32_t* dig = digs + (threadIdx.x & ~15u) * 8;
    uint32_t st2[8];
    kp_seed(j.header, j.nonce, st2);
    kp_group_hashes((const uint4*)p.dag, p.items, l1, st2[0], st2[1], lane, dig);
    __syncthreads();
    uint32_t digest[8], fin[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) digest[k] = dig[lane * 8 + k];
    kp_final(st2, digest, fin);
    if (valid) {
        uint32_t* o = p.out + (size_t)job * 16;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            o[k] = digest[k];
            o[8 + k] = fin[k];
        }
    }
}
