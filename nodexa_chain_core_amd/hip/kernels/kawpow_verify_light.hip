// KawPow light-mode batch verification for gfx950 (SURVEY K3,
// `kawpow_verify_light_batch`; BASELINE config 5).
//
// Reference behaviour: progpow::hash / verify on a light epoch context
// (src/crypto/ethash/lib/ethash/progpow.cpp:298-355, 431-495), which is what
// CheckBlockHeader pays per header (~5 ms of one CPU core at epoch 384). The
// DAG items a hash touches (64 rounds x one 2048-bit item = 4 x 512-bit items,
// each 512 dependent light-cache parents, ethash.cpp:180-251) are recomputed
// on the fly instead of reading a 4 GiB DAG — for fewer than ~10^5 headers per
// epoch that is far cheaper than generating the whole DAG.
//
// CDNA4 mapping
//   * one job (header, nonce, height) per 16-lane group, 16 jobs per 256-thread
//     workgroup; every job of a batch is independent, so a 10k-header batch is
//     ~2.5k waves — enough to cover the light-cache latency chain.
//   * per round the group needs 4 x 512-bit items; lane quad q computes item
//     4*index+q cooperatively: each lane owns 4 of the 16 mix words, the
//     parent index word mix[j%16] is broadcast inside the quad with a DPP
//     quad_perm (j%16 is a literal after unrolling by 16), and each lane
//     gathers its 16 bytes of the 64-byte parent (the light cache is <= 64 MiB
//     and stays in the 256 MiB Infinity Cache).
//   * a lane then fetches its 4 words of the 256-byte item ((l^r)%16 selects
//     the slice, owned by lane (l^r)%16) with four 16-wide shuffles.
//   * the ProgPoW program is data (64 words per period, kawpow_program_words)
//     staged per group in LDS, so jobs of any period share a launch; the
//     32-word mix of each lane lives in LDS ([group][reg][lane], conflict-free
//     for a group's uniform register index).
#include "kernel_params.h"
#include "keccak_device.hpp"

#define KL_BLOCK 256
#define KL_GROUPS (KL_BLOCK / 16)

NX_DEV uint32_t kl_fnv1(uint32_t u, uint32_t v) { return (u * 0x01000193u) ^ v; }
NX_DEV uint32_t kl_fnv1a(uint32_t h, uint32_t d) { return (h ^ d) * 0x01000193u; }
NX_DEV uint32_t kl_mod(uint32_t x, const FastMod32& f) {
    const uint32_t r = x - __umulhi(x, f.mb) * f.d;  // Barrett estimate, one correction (kernel_params.h)
    return min(r, r - f.d);
}
NX_DEV uint32_t kl_clz(uint32_t x) { return x ? (uint32_t)__builtin_clz(x) : 32u; }

NX_DEV uint32_t kl_merge(uint32_t a, uint32_t b, uint32_t kind, uint32_t rot) {
    switch (kind) {
        case 0: return a * 33u + b;
        case 1: return (a ^ b) * 33u;
        case 2: return __builtin_rotateleft32(a, rot) ^ b;
        default: return __builtin_rotateright32(a, rot) ^ b;
    }
}

NX_DEV uint32_t kl_math(uint32_t a, uint32_t b, uint32_t kind) {
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
        case 9: return kl_clz(a) + kl_clz(b);
        default: return (uint32_t)(__builtin_popcount(a) + __builtin_popcount(b));
    }
}

// Broadcast the value of lane C of each aligned quad (DPP quad_perm).
template <int C>
NX_DEV uint32_t kl_quad_bcast(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, C * 0x55, 0xf, 0xf, false);
}

// Words [4s, 4s+4) of 512-bit DAG item `index`, computed by the 4 lanes of a
// quad together (s = this lane's position in the quad).
NX_DEV uint4 kl_item512(const uint4* __restrict__ light, const FastMod32& lmod, uint32_t index, uint32_t s) {
    uint32_t m[4];
    {
        // every quad lane runs the 64-byte keccak512 seed itself (cheap next to 512 parents)
        const uint32_t li = kl_mod(index, lmod);
        uint64_t in[8], out[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v = light[(size_t)li * 4 + k];
            in[2 * k] = ((uint64_t)v.y << 32) | v.x;
            in[2 * k + 1] = ((uint64_t)v.w << 32) | v.z;
        }
        in[0] ^= index;
        keccak512_64(in, out);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t w = (s & 2) ? ((s & 1) ? out[6 + (k >> 1)] : out[4 + (k >> 1)])
                                       : ((s & 1) ? out[2 + (k >> 1)] : out[k >> 1]);
            m[k] = (k & 1) ? (uint32_t)(w >> 32) : (uint32_t)w;
        }
    }
#pragma unroll 1
    for (uint32_t j = 0; j < 512; j += 16) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            // mix[k] lives in quad lane k/4, word k%4
            uint32_t own = m[k & 3];
            uint32_t mk;
            switch (k >> 2) {
                case 0: mk = kl_quad_bcast<0>(own); break;
                case 1: mk = kl_quad_bcast<1>(own); break;
                case 2: mk = kl_quad_bcast<2>(own); break;
                default: mk = kl_quad_bcast<3>(own); break;
            }
            const uint32_t parent = kl_mod(kl_fnv1(index ^ (j + (uint32_t)k), mk), lmod);
            const uint4 v = light[(size_t)parent * 4 + s];
            m[0] = kl_fnv1(m[0], v.x);
            m[1] = kl_fnv1(m[1], v.y);
            m[2] = kl_fnv1(m[2], v.z);
            m[3] = kl_fnv1(m[3], v.w);
        }
    }
    // final keccak512 over the whole 16-word mix: gather it from the quad
    uint32_t all[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        all[k] = kl_quad_bcast<0>(m[k]);
        all[4 + k] = kl_quad_bcast<1>(m[k]);
        all[8 + k] = kl_quad_bcast<2>(m[k]);
        all[12 + k] = kl_quad_bcast<3>(m[k]);
    }
    uint64_t in[8], out[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) in[k] = ((uint64_t)all[2 * k + 1] << 32) | all[2 * k];
    keccak512_64(in, out);
    const uint64_t lo = (s & 2) ? ((s & 1) ? out[6] : out[4]) : ((s & 1) ? out[2] : out[0]);
    const uint64_t hi = (s & 2) ? ((s & 1) ? out[7] : out[5]) : ((s & 1) ? out[3] : out[1]);
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

#define KL_MIX(r) mixs[(g * 32 + (r)) * 16 + lane]

// DAG = false: items recomputed from the light cache (kawpow_verify_light).
// DAG = true : items read from the resident DAG (kawpow_verify_dag) — the same
// one-job-per-group layout, so a batch whose headers span thousands of periods
// (3 headers each) needs no per-period padding, unlike kawpow_verify_batch's
// wave-uniform 64-job slabs.
template <bool DAG>
NX_DEV void kl_verify(const KawpowLightParams& p) {
    __shared__ uint32_t l1[4096];
    __shared__ uint32_t mixs[KL_GROUPS * 32 * 16];
    __shared__ uint32_t progs[KL_GROUPS * KV_PROG_WORDS];
    for (int i = threadIdx.x; i < 4096; i += KL_BLOCK) l1[i] = p.l1[i];
    const uint32_t g = threadIdx.x >> 4;
    const uint32_t lane = threadIdx.x & 15;
    const uint32_t job = blockIdx.x * KL_GROUPS + g;
    const bool valid = job < p.num_jobs;
    const uint32_t jj = valid ? job : 0;
    {
        uint32_t pi = p.job_program[jj];
        pi = pi < p.num_programs ? pi : 0;  // host validates; never index past the table
#pragma unroll
        for (int k = 0; k < 4; ++k) progs[g * KV_PROG_WORDS + lane * 4 + k] = p.programs[(size_t)pi * KV_PROG_WORDS + lane * 4 + k];
    }
    __syncthreads();
    const uint32_t* prog = &progs[g * KV_PROG_WORDS];
    const KawpowVerifyJob j = p.jobs[jj];
    const uint4* light = (const uint4*)p.light;

    uint32_t st2[8];
    {
        uint32_t s[25];
#pragma unroll
        for (int i = 0; i < 8; ++i) s[i] = j.header[i];
        s[8] = (uint32_t)j.nonce;
        s[9] = (uint32_t)(j.nonce >> 32);
        const uint32_t pad[15] = {0x72, 0x41, 0x56, 0x45, 0x4E, 0x43, 0x4F, 0x49, 0x4E, 0x4B, 0x41, 0x57, 0x50, 0x4F, 0x57};
#pragma unroll
        for (int i = 0; i < 15; ++i) s[10 + i] = pad[i];
        keccak_f800(s);
#pragma unroll
        for (int i = 0; i < 8; ++i) st2[i] = s[i];
    }
    {
        const uint32_t z0 = kl_fnv1a(0x811c9dc5u, st2[0]);
        const uint32_t w0 = kl_fnv1a(z0, st2[1]);
        const uint32_t jsr0 = kl_fnv1a(w0, lane);
        uint32_t kz = z0, kw = w0, kj = jsr0, kc = kl_fnv1a(jsr0, lane);
        for (int r = 0; r < 32; ++r) {
            kz = 36969u * (kz & 0xffffu) + (kz >> 16);
            kw = 18000u * (kw & 0xffffu) + (kw >> 16);
            kc = 69069u * kc + 1234567u;
            kj ^= (kj << 17);
            kj ^= (kj >> 13);
            kj ^= (kj << 5);
            KL_MIX(r) = (((kz << 16) + kw) ^ kc) + kj;
        }
    }
    const uint32_t q = lane >> 2, s = lane & 3;
    for (uint32_t r = 0; r < 64; ++r) {
        const uint32_t index = kl_mod(__shfl(KL_MIX(0), (int)(r & 15), 16), p.items);
        uint4 mine;
        if constexpr (DAG) {
            // lane l = 4q+s holds words 4l..4l+3 of the 2048-bit item: one coalesced 256 B load per group
            mine = ((const uint4*)p.dag)[(size_t)index * 16 + lane];
        } else {
            mine = kl_item512(light, p.light_items, index * 4 + q, s);
        }
        // lane l merges words ((l^r)%16)*4..+3 of the 2048-bit item: owned by lane (l^r)%16
        const int src = (int)((lane ^ r) & 15);
        const uint32_t dw[4] = {(uint32_t)__shfl((int)mine.x, src, 16), (uint32_t)__shfl((int)mine.y, src, 16),
                                (uint32_t)__shfl((int)mine.z, src, 16), (uint32_t)__shfl((int)mine.w, src, 16)};
        for (int i = 0; i < 18; ++i) {
            if (i < 11) {
                const uint32_t op = prog[i];
                const uint32_t a = KL_MIX(op & 31);
                uint32_t& dst = KL_MIX((op >> 8) & 31);
                dst = kl_merge(dst, l1[a & 4095u], (op >> 16) & 3, op >> 24);
            }
            const uint32_t op = prog[11 + i];
            const uint32_t mg = prog[29 + i];
            const uint32_t v = kl_math(KL_MIX(op & 31), KL_MIX((op >> 8) & 31), (op >> 16) & 15);
            uint32_t& dst = KL_MIX(op >> 24);
            dst = kl_merge(dst, v, mg & 3, mg >> 8);
        }
        for (int i = 0; i < 4; ++i) {
            const uint32_t op = prog[47 + i];
            uint32_t& dst = KL_MIX(op & 31);
            dst = kl_merge(dst, dw[i], (op >> 8) & 3, op >> 16);
        }
    }
    uint32_t lh = 0x811c9dc5u;
    for (int r = 0; r < 32; ++r) lh = kl_fnv1a(lh, KL_MIX(r));
    uint32_t digest[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t a = __shfl(lh, k, 16);
        const uint32_t b = __shfl(lh, k + 8, 16);
        digest[k] = kl_fnv1a(kl_fnv1a(0x811c9dc5u, a), b);
    }
    uint32_t st[25];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = st2[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[8 + i] = digest[i];
    const uint32_t pad[9] = {0x72, 0x41, 0x56, 0x45, 0x4E, 0x43, 0x4F, 0x49, 0x4E};
#pragma unroll
    for (int i = 0; i < 9; ++i) st[16 + i] = pad[i];
    keccak_f800(st);
    if (valid && lane == 0) {
        uint32_t* o = p.out + (size_t)job * 16;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            o[k] = digest[k];
            o[8 + k] = st[k];
        }
    }
}

extern "C" __global__ __launch_bounds__(KL_BLOCK) void kawpow_verify_light(KawpowLightParams p) { kl_verify<false>(p); }
extern "C" __global__ __launch_bounds__(KL_BLOCK) void kawpow_verify_dag(KawpowLightParams p) { kl_verify<true>(p); }

// ---------------------------------------------------------------- wave-uniform programs
// kawpow_verify_waves: one job per 16-lane group against the resident DAG, like kawpow_verify_dag,
// but the 4 groups of a wave64 hold jobs of ONE period (p.slots, built by the host: the batch's
// KawPow rows grouped by period, 4 slots per wave, -1 = idle group). The program is then uniform
// over the wave: its op words come through scalar loads, the op and merge kinds are scalar
// branches, and the 32-word mix stays in VGPRs, addressed by uniform register moves -- where the
// LDS-mix interpreter above pays two or three dependent LDS round trips per op. A batch of 3
// headers per period idles a quarter of the groups; each job is ~64 dependent DAG rounds, so the
// launch is latency-bound and the idle groups cost nothing measurable.
typedef uint32_t kw_mix_t __attribute__((ext_vector_type(32)));

NX_DEV uint32_t kw_get(const kw_mix_t& m, uint32_t i) { return m[i & 31]; }
NX_DEV void kw_set(kw_mix_t& m, uint32_t i, uint32_t v) { m[i & 31] = v; }

// Op dispatch: one shared handler table per kernel, called per op. The op and merge kinds are
// wave-uniform, but as C++ switches they lower to scalar branch trees (~4 levels for the 11 math
// kinds, each level a compare, a branch and the structurizer's flow blocks), and those trees were
// 57 % of the kernel (profiles/README r5o: 711 -> 309 us with the kinds fixed). Branch-free VALU
// selects cost more than they save (r5g: every candidate computed, 586 against 458 us). Instead the
// kinds index 64-byte handler slots: `s_swappc_b64` into slot 4 * math + merge (math and the merge
// of its result fused, one call per op) or 44 + merge (the cache and DAG merges), and the handler
// returns with `s_setpc_b64`: two jumps per op whatever the kinds, bit-exact, 712 -> 518 us for
// the 10k fixture's two launches (r5o). tools/check_jump_slots.py checks every slot's first
// instruction in the built code object (tests/test_kernel_isa.py).
//
// Calling convention (registers pinned by the asm constraints, so the compiler moves the mix
// words in and out around each call): v61 = a, v62 = b (clobbered by the clz handler), v63 = the
// destination's old value in and the merged value out, v60 = the math result (in: the value of a
// merge-only slot), s96 = the merge rotation, s[94:95] = the target, s[98:99] = the return address,
// s97 = scratch. Every asm statement declares SCC clobbered: the dispatch's adds write it, and a
// compare the compiler had scheduled across the call would otherwise branch on a stale value.
#define KWM0 "v_add_u32_e32 v60, v61, v62\n"
#define KWM1 "v_mul_lo_u32 v60, v61, v62\n"
#define KWM2 "v_mul_hi_u32 v60, v61, v62\n"
#define KWM3 "v_min_u32_e32 v60, v61, v62\n"
#define KWM4 "v_sub_u32_e32 v60, 0, v62\n v_alignbit_b32 v60, v61, v61, v60\n"
#define KWM5 "v_alignbit_b32 v60, v61, v61, v62\n"
#define KWM6 "v_and_b32_e32 v60, v61, v62\n"
#define KWM7 "v_or_b32_e32 v60, v61, v62\n"
#define KWM8 "v_xor_b32_e32 v60, v61, v62\n"
#define KWM9 "v_ffbh_u32_e32 v60, v61\n v_min_u32_e32 v60, 32, v60\n v_ffbh_u32_e32 v62, v62\n v_min_u32_e32 v62, 32, v62\n v_add_u32_e32 v60, v60, v62\n"
#define KWM10 "v_bcnt_u32_b32 v60, v61, 0\n v_bcnt_u32_b32 v60, v62, v60\n"
#define KWG0 "v_lshl_add_u32 v63, v63, 5, v63\n v_add_u32_e32 v63, v63, v60\n"
#define KWG1 "v_xor_b32_e32 v63, v63, v60\n v_lshl_add_u32 v63, v63, 5, v63\n"
#define KWG2 "s_sub_u32 s97, 0, s96\n v_alignbit_b32 v63, v63, v63, s97\n v_xor_b32_e32 v63, v63, v60\n"
#define KWG3 "v_alignbit_b32 v63, v63, v63, s96\n v_xor_b32_e32 v63, v63, v60\n"
#define KWS(n, body) ".org .Lkwt_tab%=+(" #n ")*64\n" body "s_setpc_b64 s[98:99]\n"
#define KWS4(m, n0) KWS(n0, KWM##m KWG0) KWS(n0 + 1, KWM##m KWG1) KWS(n0 + 2, KWM##m KWG2) KWS(n0 + 3, KWM##m KWG3)

// the table, jumped over once per wave; returns its address
NX_DEV void kwt_table(uint32_t& lo, uint32_t& hi) {
    asm volatile(
        "s_getpc_b64 s[94:95]\n"
        ".Lkwt_pc%=:\n"
        "s_add_u32 %[lo], s94, .Lkwt_tab%=-.Lkwt_pc%=\n"
        "s_addc_u32 %[hi], s95, 0\n"
        "s_branch .Lkwt_end%=\n"
        ".p2align 6\n"
        ".Lkwt_tab%=:\n"
        KWS4(0, 0) KWS4(1, 4) KWS4(2, 8) KWS4(3, 12) KWS4(4, 16) KWS4(5, 20) KWS4(6, 24) KWS4(7, 28)
        KWS4(8, 32) KWS4(9, 36) KWS4(10, 40)
        KWS(44, KWG0) KWS(45, KWG1) KWS(46, KWG2) KWS(47, KWG3)
        ".org .Lkwt_tab%=+48*64\n"
        ".Lkwt_end%=:\n"
        : [lo] "=s"(lo), [hi] "=s"(hi)
        :
        : "s94", "s95", "scc");
}

// d = merge(d, math(a, b)) through fused slot 4 * min(kind, 10) + merge kind
NX_DEV uint32_t kwt_op(uint32_t lo, uint32_t hi, uint32_t a, uint32_t b, uint32_t d, uint32_t kind, uint32_t mkind,
                       uint32_t rot) {
    const uint32_t off = ((kind < 10u ? kind : 10u) * 4u + (mkind & 3u)) << 6;
    asm volatile(
        "s_add_u32 s94, %[lo], %[off]\n"
        "s_addc_u32 s95, %[hi], 0\n"
        "s_swappc_b64 s[98:99], s[94:95]\n"
        : "+{v63}"(d), "+{v62}"(b)
        : "{v61}"(a), "{s96}"(rot), [lo] "s"(lo), [hi] "s"(hi), [off] "s"(off)
        : "v60", "s94", "s95", "s97", "s98", "s99", "scc");
    return d;
}

// d = merge(d, v) through merge-only slot 44 + merge kind
NX_DEV uint32_t kwt_merge(uint32_t lo, uint32_t hi, uint32_t d, uint32_t v, uint32_t mkind, uint32_t rot) {
    const uint32_t off = (44u + (mkind & 3u)) << 6;
    asm volatile(
        "s_add_u32 s94, %[lo], %[off]\n"
        "s_addc_u32 s95, %[hi], 0\n"
        "s_swappc_b64 s[98:99], s[94:95]\n"
        : "+{v63}"(d)
        : "{v60}"(v), "{s96}"(rot), [lo] "s"(lo), [hi] "s"(hi), [off] "s"(off)
        : "s94", "s95", "s97", "s98", "s99", "scc");
    return d;
}

extern "C" __global__ __launch_bounds__(KL_BLOCK) void kawpow_verify_waves(KawpowLightParams p) {
    __shared__ uint32_t l1[4096];
    for (int i = threadIdx.x; i < 4096; i += KL_BLOCK) l1[i] = p.l1[i];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 15;
    const uint32_t g = (threadIdx.x >> 4) & 3;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (KL_BLOCK / 64) + (threadIdx.x >> 6));
    if (wave * 4 >= p.num_slots) return;  // wave-uniform: whole waves only
    const int32_t first = __builtin_amdgcn_readfirstlane(p.slots[wave * 4]);  // slot 0 of a wave is never idle
    const int32_t row = p.slots[wave * 4 + g];
    const bool valid = row >= 0;
    const uint32_t jj = (uint32_t)(valid ? row : first);
    uint32_t pi = __builtin_amdgcn_readfirstlane(p.job_program[first]);
    pi = pi < p.num_programs ? pi : 0;  // host validates; never index past the table
    const uint32_t* prog = p.programs + (size_t)pi * KV_PROG_WORDS;
    // the period's 51 op words, loaded once into SGPRs: inside the round loop every op word is a
    // literal SGPR (the loop below is unrolled), so no op waits on a scalar load -- and the LDS L1
    // lookups, which share the lgkm counter with scalar loads, no longer wait behind them either
    uint32_t pw[51];
#pragma unroll
    for (int i = 0; i < 51; ++i) pw[i] = __builtin_amdgcn_readfirstlane(prog[i]);
    const KawpowVerifyJob j = p.jobs[jj];

    uint32_t st2[8];
    {
        uint32_t s[25];
#pragma unroll
        for (int i = 0; i < 8; ++i) s[i] = j.header[i];
        s[8] = (uint32_t)j.nonce;
        s[9] = (uint32_t)(j.nonce >> 32);
        const uint32_t pad[15] = {0x72, 0x41, 0x56, 0x45, 0x4E, 0x43, 0x4F, 0x49, 0x4E, 0x4B, 0x41, 0x57, 0x50, 0x4F, 0x57};
#pragma unroll
        for (int i = 0; i < 15; ++i) s[10 + i] = pad[i];
        keccak_f800(s);
#pragma unroll
        for (int i = 0; i < 8; ++i) st2[i] = s[i];
    }
    kw_mix_t mix;
    {
        const uint32_t z0 = kl_fnv1a(0x811c9dc5u, st2[0]);
        const uint32_t w0 = kl_fnv1a(z0, st2[1]);
        const uint32_t jsr0 = kl_fnv1a(w0, lane);
        uint32_t kz = z0, kw = w0, kj = jsr0, kc = kl_fnv1a(jsr0, lane);
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            kz = 36969u * (kz & 0xffffu) + (kz >> 16);
            kw = 18000u * (kw & 0xffffu) + (kw >> 16);
            kc = 69069u * kc + 1234567u;
            kj ^= (kj << 17);
            kj ^= (kj >> 13);
            kj ^= (kj << 5);
            mix[r] = (((kz << 16) + kw) ^ kc) + kj;
        }
    }
    const uint4* dag = (const uint4*)p.dag;
    uint32_t tlo, thi;
    kwt_table(tlo, thi);
#pragma unroll 1
    for (uint32_t r = 0; r < 64; ++r) {
        const uint32_t index = kl_mod(__shfl(mix[0], (int)(r & 15), 16), p.items);
        // lane l merges words ((l^r)%16)*4..+3 of the 2048-bit item: load exactly that slice
        const uint4 d = dag[(size_t)index * 16 + ((lane ^ r) & 15)];
        // opaque per round: the op fields are decoded where they are used (SALU, next to the op)
        // instead of being hoisted out of the loop into ~150 loop-invariant SGPRs that spill
#pragma unroll
        for (int i = 0; i < 51; ++i) asm volatile("" : "+s"(pw[i]));
#pragma unroll
        for (int i = 0; i < 18; ++i) {
            if (i < 11) {
                const uint32_t op = pw[i];
                const uint32_t dst = (op >> 8) & 31;
                kw_set(mix, dst, kwt_merge(tlo, thi, kw_get(mix, dst), l1[kw_get(mix, op) & 4095u], (op >> 16) & 3, op >> 24));
            }
            const uint32_t op = pw[11 + i];
            const uint32_t mg = pw[29 + i];
            const uint32_t dst = op >> 24;
            kw_set(mix, dst, kwt_op(tlo, thi, kw_get(mix, op), kw_get(mix, op >> 8), kw_get(mix, dst), (op >> 16) & 15,
                                    mg & 3, mg >> 8));
        }
        const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t op = pw[47 + i];
            kw_set(mix, op, kwt_merge(tlo, thi, kw_get(mix, op), dw[i], (op >> 8) & 3, op >> 16));
        }
    }
    uint32_t lh = 0x811c9dc5u;
#pragma unroll
    for (int r = 0; r < 32; ++r) lh = kl_fnv1a(lh, mix[r]);
    uint32_t digest[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t a = __shfl(lh, k, 16);
        const uint32_t b = __shfl(lh, k + 8, 16);
        digest[k] = kl_fnv1a(kl_fnv1a(0x811c9dc5u, a), b);
    }
    uint32_t st[25];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = st2[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[8 + i] = digest[i];
    const uint32_t pad[9] = {0x72, 0x41, 0x56, 0x45, 0x4E, 0x43, 0x4F, 0x49, 0x4E};
#pragma unroll
    for (int i = 0; i < 9; ++i) st[16 + i] = pad[i];
    keccak_f800(st);
    if (valid && lane == 0) {
        uint32_t* o = p.out + (size_t)row * 16;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            o[k] = digest[k];
            o[8 + k] = st[k];
        }
    }
}

