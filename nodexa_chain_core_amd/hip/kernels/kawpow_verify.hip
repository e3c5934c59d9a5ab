// KawPow batch verification kernel for gfx950 — one launch covers every
// ProgPoW period in the batch (BASELINE config 5).
//
// The search kernel bakes one period's program into the code; a batch of
// headers from a chain segment spans many periods (3 blocks each), so here the
// program is data: the host materialises each distinct period's op list
// (csrc/pow/kawpow.cpp make_kawpow_program) and sorts jobs so that every
// wave64 (4 hashes x 16 lanes, 64 jobs walked by the wave) shares one period.
// The op fields are then wave-uniform (readfirstlane), so the 32-word mix (in
// LDS, [wave][group][reg][lane]) is addressed with uniform offsets instead of a
// divergent waterfall. Each group walks 16 jobs of its slab, so this layout
// suits periods with many jobs; a header batch (3 headers per period) uses
// kawpow_verify_waves (kawpow_verify_light.hip) instead.
#include "kernel_params.h"
#include "keccak_device.hpp"

// Program encoding, 64 u32 per period:
//   [0..10]  cache op i : src | dst << 8 | merge_kind << 16 | rot << 24
//   [11..28] math op i  : src1 | src2 << 8 | math_kind << 16 | dst << 24
//   [29..46] math merge : merge_kind | rot << 8
//   [47..50] dag merge  : dst | merge_kind << 8 | rot << 16
// (KV_PROG_WORDS and KawpowVerifyParams live in kernel_params.h)

NX_DEV uint32_t kv_fnv1a(uint32_t h, uint32_t d) { return (h ^ d) * 0x01000193u; }
NX_DEV uint32_t kv_fastmod(uint32_t x, const FastMod32& f) {
    const uint32_t t = __umulhi(x, f.m);
    const uint32_t q = (t + ((x - t) >> 1)) >> (f.s - 1);
    return x - q * f.d;
}
NX_DEV uint32_t kv_clz(uint32_t x) { return x ? (uint32_t)__builtin_clz(x) : 32u; }

NX_DEV uint32_t kv_merge(uint32_t a, uint32_t b, uint32_t kind, uint32_t rot) {
    switch (kind) {
        case 0: return a * 33u + b;
        case 1: return (a ^ b) * 33u;
        case 2: return __builtin_rotateleft32(a, rot) ^ b;
        default: return __builtin_rotateright32(a, rot) ^ b;
    }
}

NX_DEV uint32_t kv_math(uint32_t a, uint32_t b, uint32_t kind) {
    switch (kind) {
        case 0: return a + b;
        case 1: return a * b;
        case 2: return __umulhi(a, b);
        case 3: return min(a, b);
        case 4: return __builtin_rotateleft32(a, b);
        case 5: return __builtin_rotateright32(a, b);
        case 6: return a & b;
        case 7: return a | b;
        case 8: return a ^ b;
        case 9: return kv_clz(a) + kv_clz(b);
        default: return (uint32_t)(__builtin_popcount(a) + __builtin_popcount(b));
    }
}

// The mix lives in LDS: [wave][group(4)][reg(32)][lane(16)] so a uniform-register
// access by the 64 threads of a wave touches 64 consecutive words (conflict-free).
#define KV_MIX(r) mixs[(wslot * 32 + (r)) * 64 + tl]

NX_DEV void kv_seed(const uint32_t header[8], uint64_t nonce, uint32_t st2[8]) {
    uint32_t s[25];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = header[i];
    s[8] = (uint32_t)nonce;
    s[9] = (uint32_t)(nonce >> 32);
    const uint32_t pad[15] = {0x72, 0x41, 0x56, 0x45, 0x4E, 0x43, 0x4F, 0x49, 0x4E, 0x4B, 0x41, 0x57, 0x50, 0x4F, 0x57};
#pragma unroll
    for (int i = 0; i < 15; ++i) s[10 + i] = pad[i];
    keccak_f800(s);
#pragma unroll
    for (int i = 0; i < 8; ++i) st2[i] = s[i];
}

extern "C" __global__ __launch_bounds__(256) void kawpow_verify_batch(KawpowVerifyParams p) {
    __shared__ uint32_t l1[4096];
    __shared__ uint32_t mixs[4 * 32 * 64];  // 4 waves x 32 regs x 64 threads
    {
        const uint4* src = (const uint4*)p.dag;
        uint4* dst = (uint4*)l1;
        for (int i = threadIdx.x; i < 1024; i += 256) dst[i] = src[i];
    }
    __syncthreads();
    const uint32_t tl = threadIdx.x & 63;  // thread within wave
    const uint32_t wslot = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 15;
    const uint32_t job = blockIdx.x * 256 + threadIdx.x;
    const uint32_t slab = __builtin_amdgcn_readfirstlane(job >> 6);
    // num_jobs is a multiple of 64, so this exit is wave-uniform; waves past the
    // last slab must not index job_program (it has num_jobs / 64 entries).
    if (slab >= (p.num_jobs >> 6)) return;
    const uint32_t* prog = p.programs + (size_t)p.job_program[slab] * KV_PROG_WORDS;
    const bool valid = job < p.num_jobs;
    const KawpowVerifyJob j = p.jobs[valid ? job : 0];
    uint32_t st2[8];
    kv_seed(j.header, j.nonce, st2);
    uint32_t digest[8];
    for (uint32_t h = 0; h < 16; ++h) {
        const uint32_t s0 = __shfl(st2[0], (int)h, 16);
        const uint32_t s1 = __shfl(st2[1], (int)h, 16);
        const uint32_t z = kv_fnv1a(0x811c9dc5u, s0);
        const uint32_t w = kv_fnv1a(z, s1);
        const uint32_t jsr0 = kv_fnv1a(w, lane);
        uint32_t kz = z, kw = w, kj = jsr0, kc = kv_fnv1a(jsr0, lane);
        for (int r = 0; r < 32; ++r) {
            kz = 36969u * (kz & 0xffffu) + (kz >> 16);
            kw = 18000u * (kw & 0xffffu) + (kw >> 16);
            kc = 69069u * kc + 1234567u;
            kj ^= (kj << 17);
            kj ^= (kj >> 13);
            kj ^= (kj << 5);
            KV_MIX(r) = (((kz << 16) + kw) ^ kc) + kj;
        }
        for (uint32_t r = 0; r < 64; ++r) {
            const uint32_t src = __shfl(KV_MIX(0), (int)(r & 15), 16);
            const uint32_t index = kv_fastmod(src, p.items);
            const uint4 d = ((const uint4*)p.dag)[(size_t)index * 16 + ((lane ^ r) & 15)];
            for (int i = 0; i < 18; ++i) {
                if (i < 11) {
                    const uint32_t op = __builtin_amdgcn_readfirstlane(prog[i]);
                    const uint32_t a = KV_MIX(op & 31);
                    uint32_t& dst = KV_MIX((op >> 8) & 31);
                    dst = kv_merge(dst, l1[a & 4095u], (op >> 16) & 3, op >> 24);
                }
                const uint32_t op = __builtin_amdgcn_readfirstlane(prog[11 + i]);
                const uint32_t mg = __builtin_amdgcn_readfirstlane(prog[29 + i]);
                const uint32_t v = kv_math(KV_MIX(op & 31), KV_MIX((op >> 8) & 31), (op >> 16) & 15);
                uint32_t& dst = KV_MIX(op >> 24);
                dst = kv_merge(dst, v, mg & 3, mg >> 8);
            }
            const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
            for (int i = 0; i < 4; ++i) {
                const uint32_t op = __builtin_amdgcn_readfirstlane(prog[47 + i]);
                uint32_t& dst = KV_MIX(op & 31);
                dst = kv_merge(dst, dw[i], (op >> 8) & 3, op >> 16);
            }
        }
        uint32_t lh = 0x811c9dc5u;
        for (int r = 0; r < 32; ++r) lh = kv_fnv1a(lh, KV_MIX(r));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t a = __shfl(lh, k, 16);
            const uint32_t b = __shfl(lh, k + 8, 16);
            const uint32_t v = kv_fnv1a(kv_fnv1a(0x811c9dc5u, a), b);
            if (h == lane) digest[k] = v;
        }
    }
    uint32_t s[25];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = st2[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[8 + i] = digest[i];
    const uint32_t pad[9] = {0x72, 0x41, 0x56, 0x45, 0x4E, 0x43, 0x4F, 0x49, 0x4E};
#pragma unroll
    for (int i = 0; i < 9; ++i) s[16 + i] = pad[i];
    keccak_f800(s);
    if (valid) {
        uint32_t* o = p.out + (size_t)job * 16;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            o[k] = digest[k];
            o[8 + k] = s[k];
        }
    }
}
