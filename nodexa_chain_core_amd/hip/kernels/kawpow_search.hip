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
//     4 hashes side by side. Each thread owns one nonce: it computes that
//     nonce's keccak-f800 seed, then its group walks the group's 16 nonces one
//     after another (the keccak cost is paid once per nonce, not 16x).
//   * the 32 mix registers are named scalars (m0..m31): with the program baked
//     in, every index is a literal and the state never leaves VGPRs.
//   * the 16 KiB L1 (first 64 DAG items) sits in LDS; cache ops are
//     ds_read_b32 with a 12-bit masked address.
//   * each round's 256-byte DAG item is one coalesced 16 B/lane load by the
//     group (lane l takes words ((l^r)%16)*4..+3), issued at round start and
//     consumed at round end, so the 29 cache/math ops hide its HBM latency.
//   * the round's item index is broadcast from lane r%16 with ds_bpermute
//     (__shfl, width 16) and reduced with a FastMod32 multiply-shift.
#include "kernel_params.h"
#include "keccak_device.hpp"

#ifndef KAWPOW_PROGRAM_HEADER
#define KAWPOW_PROGRAM_HEADER "kawpow_program_default.inc"
#endif
#include KAWPOW_PROGRAM_HEADER

// Tuning knobs (compile-time; ops/jit.py passes them as -D variants):
//   KP_MIN_WAVES  minimum waves per SIMD for __launch_bounds__ (caps VGPRs)
//   KP_NT_DAG     non-temporal DAG loads (the 4 GiB DAG has no L2 reuse)
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
#define KP_DAG_LOAD(p) kp_dag_load(p)

#define KP_REGS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) \
    X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31)

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

// Mix of one hash for the calling lane; returns this lane's FNV lane-hash.
// `seed0/seed1` are the hash's keccak seed words, identical across the group.
NX_DEV uint32_t kp_hash_lane(const uint4* __restrict__ dag, const FastMod32& items, const uint32_t* l1,
                             uint32_t seed0, uint32_t seed1, uint32_t lane) {
    const uint32_t z = kp_fnv1a(0x811c9dc5u, seed0);
    const uint32_t w = kp_fnv1a(z, seed1);
    const uint32_t jsr = kp_fnv1a(w, lane);
    KpKiss rng{z, w, jsr, kp_fnv1a(jsr, lane)};
#define KP_DECL(i) uint32_t m##i = rng.next();
    KP_REGS(KP_DECL)
#undef KP_DECL

#pragma unroll 1
    for (uint32_t r = 0; r < 64; ++r) {
        const uint32_t src = __shfl(m0, (int)(r & 15), 16);
        const uint32_t index = kp_fastmod(src, items);
        const uint4 d = KP_DAG_LOAD(dag + (size_t)index * 16 + ((lane ^ r) & 15));
        KAWPOW_PROGRAM(l1);
        KAWPOW_DAG_MERGE(d);
    }
    uint32_t h = 0x811c9dc5u;
#define KP_RED(i) h = kp_fnv1a(h, m##i);
    KP_REGS(KP_RED)
#undef KP_RED
    return h;
}

extern "C" __global__ KP_BOUNDS void kawpow_search(KawpowSearchParams p) {
    __shared__ uint32_t l1[4096];
    {
        const uint4* src = (const uint4*)p.dag;
        uint4* dst = (uint4*)l1;
#pragma unroll
        for (int i = threadIdx.x; i < 1024; i += NODEXA_KAWPOW_BLOCK) dst[i] = src[i];
    }
    __syncthreads();

    const uint32_t lane = threadIdx.x & 15;
    const uint64_t nonce = p.start_nonce + (uint64_t)blockIdx.x * NODEXA_KAWPOW_BLOCK + threadIdx.x;
    uint32_t st2[8];
    kp_seed(p.header, nonce, st2);

    uint32_t digest[8];
#pragma unroll 1
    for (uint32_t h = 0; h < 16; ++h) {
        const uint32_t s0 = __shfl(st2[0], (int)h, 16);
        const uint32_t s1 = __shfl(st2[1], (int)h, 16);
        const uint32_t lh = kp_hash_lane((const uint4*)p.dag, p.items, l1, s0, s1, lane);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t a = __shfl(lh, k, 16);
            const uint32_t b = __shfl(lh, k + 8, 16);
            const uint32_t v = kp_fnv1a(kp_fnv1a(0x811c9dc5u, a), b);
            if (h == lane) digest[k] = v;
        }
    }

    uint32_t fin[8];
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
    uint32_t st2[8];
    kp_seed(j.header, j.nonce, st2);
    uint32_t digest[8];
#pragma unroll 1
    for (uint32_t h = 0; h < 16; ++h) {
        const uint32_t s0 = __shfl(st2[0], (int)h, 16);
        const uint32_t s1 = __shfl(st2[1], (int)h, 16);
        const uint32_t lh = kp_hash_lane((const uint4*)p.dag, p.items, l1, s0, s1, lane);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t a = __shfl(lh, k, 16);
            const uint32_t b = __shfl(lh, k + 8, 16);
            const uint32_t v = kp_fnv1a(kp_fnv1a(0x811c9dc5u, a), b);
            if (h == lane) digest[k] = v;
        }
    }
    uint32_t fin[8];
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
