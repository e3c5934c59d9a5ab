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
//   * measured (profiles/README.md): the kernel is VALU-issue bound, not HBM
//     bound — ~2k wave64 integer VALU instructions per hash at 4 cycles each
//     saturate the SIMDs at ~270 MH/s while the 16 KiB/hash of DAG gathers
//     runs at ~4.4 TB/s. Doubling gathers in flight (KP_HASHES=2/4) did not
//     help; every VALU op removed from the round did. So the tuned variant
//     (ops/jit.py TUNED_DEFINES) spends its effort on instruction count:
//       - rounds unrolled by 16 so the item-index broadcast from lane r%16 is
//         one DPP row_newbcast (no ds_bpermute / address math),
//       - a 5-op Barrett modulo for the item index,
//       - raw-buffer DAG loads with a 32-bit byte offset,
//       - the L1 replicated 4x in LDS so each of the 11 cache lookups needs a
//         single v_lshlrev_b16 for its address (two 768-thread workgroups, 6
//         waves/SIMD, within the 160 KiB LDS).
//   * the mix registers are arrays subscripted only by literals (the emitted
//     program bakes every index in), so they are scalarised into VGPRs.
//   * everything not needed inside the round loop leaves the VGPR file: each
//     hash's 8 digest words are parked in the 8 VGPRs of the lane that owns it,
//     and the keccak state words 2..7 are recomputed for the final absorb
//     instead of being held live.
//   * each round's 256-byte DAG item is one coalesced 16 B/lane load by the
//     group (lane l takes words ((l^r)%16)*4..+3).
#include "kernel_params.h"
#include "keccak_device.hpp"

// Ceiling microbenchmark (tools/kawpow_sweep.py, profiles/r4a): compile one class of the period's
// ops out of the real kernel at the shipping occupancy. KP_SKEL_NOMATH keeps the DAG gather chain
// and the 11 L1 lookups (+ their merges) per round, KP_SKEL_NOCACHE the gathers and the 18 math
// ops, KP_SKEL_GATHER only the gather chain and its merge. Never bit-exact; never shipped.
#if defined(KP_SKEL_NOMATH) || defined(KP_SKEL_GATHER)
#define KP_MATH_OP(...)
#endif
#if defined(KP_SKEL_NOCACHE) || defined(KP_SKEL_GATHER)
#define KP_CACHE_OP(...)
#endif
#ifndef KAWPOW_PROGRAM_HEADER
#define KAWPOW_PROGRAM_HEADER "kawpow_program_default.inc"
#endif
#include KAWPOW_PROGRAM_HEADER

// Tuning knobs (compile-time; ops/jit.py passes them as -D variants). The variants measured and
// lost were removed after round 3 (profiles/README r4a: KP_L1G, KP_BUFFER, KP_MUL33_SHIFT,
// KP_DIGEST_GLOBAL, KP_FASTMOD24, KP_PRIO and the loop without DPP broadcasts); the search is
// bounded by its own gather + L1-lookup skeleton (the KP_SKEL_* ceiling above), not by a knob.
//   KP_HASHES     hashes interleaved per 16-lane group (1, 2, 4 or 8)
//   KP_MIN_WAVES  minimum waves per SIMD for __launch_bounds__ (caps VGPRs)
//   KP_NT_DAG     non-temporal DAG loads (the 4 GiB DAG has no L2 reuse)
//   KP_SCHED_FENCE scheduling barriers around each round's cache/math program, so the DAG
//                 gather issued at the top of the round is consumed only at its end
#ifndef KP_HASHES
#define KP_HASHES 2
#endif
#if (16 % KP_HASHES) != 0
#error "KP_HASHES must divide 16"
#endif
//   KP_BLOCK      threads per workgroup (the host launcher reads it back from
//                 the kernel's max-threads attribute)
//   KP_DPP        (always on; accepted for compatibility) rounds unrolled by 16, the item index
//                 broadcast by DPP row_newbcast
//   KP_BARRETT    5-op Barrett modulo for the item index
//   KP_SBUFFER    structured-buffer DAG loads (item index x 256 B stride)
//   KP_PTR64      (instead of KP_SBUFFER) 64-bit item addresses, one v_mad_u64_u32: DAGs >= 4 GiB
//   KP_L1X4       L1 replicated 4x in LDS (64 KiB) so an L1 address is one
//                 16-bit shift: ((x << 2) & 0xffff) reads l1[x % 4096]
// Digests: each finished hash's 8 digest words go straight to the lane that owns the hash's
// nonce (8 DPP broadcasts + 8 selects per hash, 8 VGPRs), so the workgroup's LDS is only the L1
// table and two 768-thread groups share a CU. (The 32 B/nonce LDS-digest form measured equal on
// the >4 GiB pointer path, 269.8 vs 269.3 MH/s at epoch 390, profiles r4b, and was removed.)
#ifndef KP_BLOCK
#define KP_BLOCK NODEXA_KAWPOW_BLOCK
#endif

#ifdef KP_MIN_WAVES
#define KP_BOUNDS __launch_bounds__(KP_BLOCK, KP_MIN_WAVES)
#else
#define KP_BOUNDS __launch_bounds__(KP_BLOCK)
#endif

#ifdef KP_L1X4
#define KP_L1_WORDS 16384
// v_lshlrev_b16 writes the low half and zeroes the high half of the VGPR, so
// the shifted value is directly a byte offset < 64 KiB into the 4 copies.
NX_DEV uint32_t kp_l1_read(const uint32_t* l1, uint32_t x) {
    uint32_t off;
    asm("v_lshlrev_b16 %0, 2, %1" : "=v"(off) : "v"(x));
    return *(const uint32_t*)((const char*)l1 + off);
}
#define KP_L1(l1, x) kp_l1_read((l1), (x))
#else
#define KP_L1_WORDS 4096
#define KP_L1(l1, x) (l1)[(x) & 4095u]
#endif

// LDS copy of the L1 (first 16 KiB of the DAG), KP_L1_WORDS / 4096 times.
NX_DEV void kp_fill_l1(uint32_t* l1, const void* dag) {
    const uint4* src = (const uint4*)dag;
    uint4* dst = (uint4*)l1;
#pragma unroll
    for (int i = threadIdx.x; i < KP_L1_WORDS / 4; i += KP_BLOCK) dst[i] = src[i & 1023];
}
typedef uint32_t kp_u32x4 __attribute__((ext_vector_type(4)));
NX_DEV uint4 kp_dag_load(const uint4* p) {
#ifdef KP_NT_DAG
    const kp_u32x4 v = __builtin_nontemporal_load((const kp_u32x4*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}

// x*33 for the merge ops: the compiler's v_mad_u64_u32 for `a*33 + b` beats a shift-add
// (profiles/README r2b).
NX_DEV uint32_t kp_mul33(uint32_t a) { return a * 33u; }

NX_DEV uint32_t kp_clz(uint32_t x) { return x ? (uint32_t)__builtin_clz(x) : 32u; }
NX_DEV uint32_t kp_fnv1a(uint32_t h, uint32_t d) { return (h ^ d) * 0x01000193u; }
NX_DEV uint32_t kp_fastmod(uint32_t x, const FastMod32& f) {
#if defined(KP_BARRETT)
    // q' = floor(x * floor(2^32/d) / 2^32) is q or q-1, so r' < 2d and one
    // unsigned min(r', r'-d) finishes it (r'-d wraps high when r' < d).
    const uint32_t r = x - __umulhi(x, f.mb) * f.d;
    return min(r, r - f.d);
#else
    const uint32_t t = __umulhi(x, f.m);
    const uint32_t q = (t + ((x - t) >> 1)) >> (f.s - 1);
    return x - q * f.d;
#endif
}

// DAG item access: structured-buffer loads (one V# below 4 GiB, two from 4 GiB up); the 64-bit
// pointer form is kept for the untuned template.
#if defined(KP_SBUFFER)
// Structured-buffer addressing: vindex = item, stride 256 B in the V#, voffset = the lane's
// 16-byte slice: one buffer_load_dwordx4 idxen offen per round and no address VALU at all
// (a raw-buffer form needed one v_lshl_add): +1.1 % at epoch 384 (profiles/r1s_kawpow). The
// hardware forms index*stride+offset in 32 bits, so it is for DAGs < 4 GiB
// (measured: not bit-exact at epoch 390). clang has no struct-buffer builtin, so the LLVM
// intrinsic is bound by name (the compiler still tracks its vmcnt like any other load).
typedef int32_t kp_i32x4 __attribute__((ext_vector_type(4)));
__device__ kp_i32x4 kp_struct_load(kp_i32x4 rsrc, int vindex, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.buffer.load.v4i32");
typedef kp_i32x4 kp_dag_t;
NX_DEV kp_dag_t kp_dag_handle(const void* dag) {
    const uint64_t base = (uint64_t)dag;
    kp_i32x4 r;
    r.x = (int32_t)(uint32_t)base;
    r.y = (int32_t)(((uint32_t)(base >> 32) & 0xffffu) | (256u << 16));  // stride 256 B
    r.z = -1;                                                             // num_records: no clamp
    r.w = 0x00020000;                                                     // DATA_FORMAT 32
    return r;
}
NX_DEV uint4 kp_dag_item(kp_dag_t dag, uint32_t index, uint32_t part) {
#ifdef KP_NT_DAG
    const int aux = 2;
#else
    const int aux = 0;
#endif
    const kp_i32x4 v = kp_struct_load(dag, (int)index, (int)(part << 4), 0, aux);
    return make_uint4((uint32_t)v.x, (uint32_t)v.y, (uint32_t)v.z, (uint32_t)v.w);
}
#else
typedef const uint4* kp_dag_t;
NX_DEV kp_dag_t kp_dag_handle(const void* dag) { return (const uint4*)dag; }
NX_DEV uint4 kp_dag_item(kp_dag_t dag, uint32_t index, uint32_t part) {
    return kp_dag_load(dag + (size_t)index * 16 + part);
}
#endif
#if defined(KP_PTR64)
// DAGs of 4 GiB or more (epochs >= 385): MUBUF offsets are 32-bit, so the item address is a 64-bit
// VGPR pair: one v_mad_u64_u32 (index * 256 + dag; dag an SGPR pair, 256 in a VGPR: one
// constant-bus read on gfx9) and one v_or for the lane's 16-byte slice (lane ^ J) * 16, which
// never carries: dag is 256-byte aligned. Measured at epoch 390 (profiles/r6_dag_over_4g):
// +1.7 % over the 512-thread pointer form; the plain C pointer form at 768 threads hoists the 16
// per-round 64-bit slice bases (32 VGPRs) and spills; a second V# for items >= 2^24 costs a second
// load instruction per round (-9 %: the gather is address-bound); a branch in the round (either
// V# per wave) spills the mix.
typedef uint64_t kp_dag_p64;
NX_DEV kp_dag_p64 kp_dag_handle_p64(const void* dag) { return (uint64_t)dag; }
typedef __attribute__((address_space(1))) const kp_u32x4 kp_gu32x4;
template <int J>
NX_DEV uint4 kp_dag_item_p64(kp_dag_p64 dag, uint32_t index, uint32_t lane16) {
    uint64_t a, carry;
    const uint32_t k256 = 256u;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(a), "=s"(carry) : "v"(index), "v"(k256), "s"(dag));
    const uint32_t lo = (uint32_t)a | (lane16 ^ (uint32_t)(J << 4));
    kp_gu32x4* ptr = (kp_gu32x4*)((a & 0xffffffff00000000ull) | lo);
#ifdef KP_NT_DAG
    const kp_u32x4 v = __builtin_nontemporal_load(ptr);
#else
    const kp_u32x4 v = *ptr;
#endif
    return make_uint4(v.x, v.y, v.z, v.w);
}
#define KP_DAG kp_dag_p64
#define KP_DAG_HANDLE kp_dag_handle_p64
#define KP_DAG_ITEM_J(dag, index, part, J) kp_dag_item_p64<J>((dag), (index), (part ^ (uint32_t)J) << 4)
#else
#define KP_DAG kp_dag_t
#define KP_DAG_HANDLE kp_dag_handle
#define KP_DAG_ITEM_J(dag, index, part, J) kp_dag_item((dag), (index), (part))
#endif

// Broadcast lane j of each 16-lane row: DPP row_newbcast (one VALU op, no LDS
// round trip) when the round index is a compile-time constant.
template <int J>
NX_DEV uint32_t kp_bcast(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + J, 0xf, 0xf, false);
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
// digest words go to `own` of the lane that owns the hash (8 DPP broadcasts).
// One ProgPoW round with the round index known mod 16 (J): the item index comes
// from lane J of the row via DPP and the lane's 16-byte slice is lane ^ J.
template <int J>
NX_DEV void kp_round_c(uint32_t (&mx)[KP_HASHES][32], const KP_DAG& dag,
                       const FastMod32& items, const uint32_t* l1, uint32_t lane) {
    uint4 d[KP_HASHES];
    const uint32_t part = lane ^ (uint32_t)J;
#pragma unroll
    for (int k = 0; k < KP_HASHES; ++k) d[k] = KP_DAG_ITEM_J(dag, kp_fastmod(kp_bcast<J>(mx[k][0]), items), part, J);
#ifdef KP_SCHED_FENCE
    // Keep the round's DAG merge after the whole cache/math program: left alone, the register-
    // pressure scheduler pulls the merge (and its vmcnt wait) into the middle of the program, so
    // a third of the round's work waits behind a ~1 us HBM gather instead of hiding it.
    __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
    for (int k = 0; k < KP_HASHES; ++k) KAWPOW_PROGRAM(l1, mx[k]);
#ifdef KP_SCHED_FENCE
    __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
    for (int k = 0; k < KP_HASHES; ++k) KAWPOW_DAG_MERGE(d[k], mx[k]);
}

NX_DEV void kp_group_hashes(const KP_DAG& dag, const FastMod32& items, const uint32_t* l1,
                            uint32_t st0, uint32_t st1, uint32_t lane, uint32_t (&own)[8]) {
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
        // 64 rounds = 4 x 16 with the round index mod 16 baked into each copy
#pragma unroll 1
        for (uint32_t rr = 0; rr < 64; rr += 16) {
            kp_round_c<0>(mx, dag, items, l1, lane);   kp_round_c<1>(mx, dag, items, l1, lane);
            kp_round_c<2>(mx, dag, items, l1, lane);   kp_round_c<3>(mx, dag, items, l1, lane);
            kp_round_c<4>(mx, dag, items, l1, lane);   kp_round_c<5>(mx, dag, items, l1, lane);
            kp_round_c<6>(mx, dag, items, l1, lane);   kp_round_c<7>(mx, dag, items, l1, lane);
            kp_round_c<8>(mx, dag, items, l1, lane);   kp_round_c<9>(mx, dag, items, l1, lane);
            kp_round_c<10>(mx, dag, items, l1, lane);  kp_round_c<11>(mx, dag, items, l1, lane);
            kp_round_c<12>(mx, dag, items, l1, lane);  kp_round_c<13>(mx, dag, items, l1, lane);
            kp_round_c<14>(mx, dag, items, l1, lane);  kp_round_c<15>(mx, dag, items, l1, lane);
        }
#pragma unroll
        for (int k = 0; k < KP_HASHES; ++k) {
            uint32_t lh = 0x811c9dc5u;
#pragma unroll
            for (int i = 0; i < 32; ++i) lh = kp_fnv1a(lh, mx[k][i]);
            // digest[j] = fnv1a(fnv1a(basis, lane_hash[j]), lane_hash[j + 8]); lanes 0..7 own j
            const uint32_t hi = __shfl(lh, (int)(lane + 8), 16);
            // lanes 0..7 hold the digest words; lane h0+k keeps all 8 of them
            const uint32_t word = kp_fnv1a(kp_fnv1a(0x811c9dc5u, lh), hi);
            const bool mine = lane == h0 + (uint32_t)k;
            // every lane runs the (convergent) broadcasts; only the owner keeps them
            const uint32_t b0 = kp_bcast<0>(word), b1 = kp_bcast<1>(word), b2 = kp_bcast<2>(word),
                           b3 = kp_bcast<3>(word), b4 = kp_bcast<4>(word), b5 = kp_bcast<5>(word),
                           b6 = kp_bcast<6>(word), b7 = kp_bcast<7>(word);
            own[0] = mine ? b0 : own[0];
            own[1] = mine ? b1 : own[1];
            own[2] = mine ? b2 : own[2];
            own[3] = mine ? b3 : own[3];
            own[4] = mine ? b4 : own[4];
            own[5] = mine ? b5 : own[5];
            own[6] = mine ? b6 : own[6];
            own[7] = mine ? b7 : own[7];
        }
    }
}

extern "C" __global__ KP_BOUNDS void kawpow_search(KawpowSearchParams p) {
    __shared__ uint32_t l1[KP_L1_WORDS];
    __shared__ uint32_t stale_word;
    uint32_t* stale = &stale_word;
    if (blockDim.x != KP_BLOCK) return;  // launched with the wrong block: no shares rather than bad ones
    if (threadIdx.x == 0) {
        // one uncached read of the host-mapped generation word per workgroup, overlapped with the
        // L1 fill below: a template change stops queued work within one workgroup's lifetime
        uint32_t s = 0;
        if (p.gen_word) s = __hip_atomic_load(p.gen_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != p.generation;
        *stale = s;
        if (s) atomicAdd(&p.results->skipped, 1u);
    }
    kp_fill_l1(l1, p.dag);
    __syncthreads();
    const uint32_t is_stale = *stale;
    if (is_stale) return;  // uniform over the workgroup

    const uint32_t lane = threadIdx.x & 15;
    const uint64_t nonce = p.start_nonce + (uint64_t)blockIdx.x * KP_BLOCK + threadIdx.x;
    uint32_t digest[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    {
        uint32_t st2[8];
        kp_seed(p.header, nonce, st2);
        kp_group_hashes(KP_DAG_HANDLE(p.dag), p.items, l1, st2[0], st2[1], lane, digest);
    }
    uint32_t st2[8], fin[8];
    // recomputed: cheaper than 6 VGPRs held across the mix loop. The nonce goes through an empty
    // asm so the compiler cannot CSE this keccak with the first one (it would keep those results
    // live across the whole hash loop and spill them).
    uint32_t nlo = (uint32_t)nonce, nhi = (uint32_t)(nonce >> 32);
    asm volatile("" : "+v"(nlo), "+v"(nhi));
    kp_seed(p.header, ((uint64_t)nhi << 32) | nlo, st2);
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
    __shared__ uint32_t l1[KP_L1_WORDS];
    if (blockDim.x != KP_BLOCK) return;
    kp_fill_l1(l1, p.dag);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 15;
    const uint32_t job = blockIdx.x * KP_BLOCK + threadIdx.x;
    const bool valid = job < p.num_jobs;
    const KawpowVerifyJob j = p.jobs[valid ? job : 0];
    uint32_t st2[8], digest[8] = {0, 0, 0, 0, 0, 0, 0, 0}, fin[8];
    kp_seed(j.header, j.nonce, st2);
    kp_group_hashes(KP_DAG_HANDLE(p.dag), p.items, l1, st2[0], st2[1], lane, digest);
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
