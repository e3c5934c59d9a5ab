// Equihash(200,9) Wagner solver for gfx950 (new; the reference has no
// Equihash — SURVEY §0.4 / Appendix D). CPU golden model: csrc/pow/equihash.cpp.
//
// Data layout (per solver instance = one header/nonce; blockIdx.y = instance):
//   digit d_j = bits [20j, 20j+20) of the 200-bit leaf string (big-endian),
//   a row of level r has d_0..d_{r-1} == 0 and lives in bucket  d_r >> 8
//   (4096 buckets x EQ_CAP slots); the low 8 bits of d_r select the
//   collision sub-bucket inside the workgroup.
//   hash table  [2][inst][4096][EQ_CAP][8] u32: word 0 = the row's ref (copied to
//               `refs` when the next round stages it), words 1..7 = the 224-bit
//               big-endian row (double-buffered across levels);
//   refs        [inst][9][4096][EQ_CAP] u32: level 0 = leaf index, level r>0 =
//               (parent bucket << 20 | slot a << 10 | slot b) into level r-1;
//   counts      [inst][10][4096] u32 bucket fill (atomics), memset per solve.
//
// Round kernel (one 256-thread workgroup per bucket, 4096 x instances
// workgroups — many times the 256 CUs): the bucket's rows are staged in LDS,
// chained by their 8-bit sub-digit with LDS atomics, every pair inside a
// chain is XORed in registers, rows whose remaining bits vanish are dropped
// (they only produce duplicate indices), and survivors are appended to their
// next-level bucket with one global atomic each. A level is ~2.1M rows x 32 B
// (67 MB), so one solver instance's live set sits in the 256 MiB Infinity Cache.
#include "equihash_device.hpp"  // BLAKE2b, digits, row XOR (shared with equihash_ps.hip)

#define EQ_BLOCK 256

NX_DEV size_t eq_hidx(const EquihashDev& p, int buf, uint32_t inst, uint32_t bucket, uint32_t slot) {
    return ((((size_t)buf * p.num_inst + inst) * EQ_BUCKETS + bucket) * EQ_CAP + slot) * EQ_WORDS;
}
NX_DEV size_t eq_ridx(const EquihashDev& p, uint32_t inst, int level, uint32_t bucket, uint32_t slot) {
    return (((size_t)inst * EQ_LEVELS + level) * EQ_BUCKETS + bucket) * EQ_CAP + slot;
}
NX_DEV uint32_t* eq_count(const EquihashDev& p, uint32_t inst, int level) {
    return p.counts + ((size_t)inst * (EQ_LEVELS + 1) + level) * EQ_BUCKETS * EQ_MAX_BANKS;
}

// Append one row to bucket `nb`: bank = blockIdx.x % banks owns slots
// [bank*per, (bank+1)*per). Returns the slot index or EQ_CAP when full.
NX_DEV uint32_t eq_alloc_slot(const EquihashDev& p, uint32_t* cnt, uint32_t nb) {
    const uint32_t bank = blockIdx.x & (p.banks - 1);
    const uint32_t per = EQ_CAP / p.banks;
    const uint32_t local = atomicAdd(&cnt[nb * EQ_MAX_BANKS + bank], 1u);
    return local < per ? bank * per + local : EQ_CAP;
}

// Gather the rows of (level, bucket) from every bank into LDS order 0..n-1;
// sid[i] = the row's slot index inside the bucket (what refs encode).
// Ends with a __syncthreads(); returns n.
// LDS row layout: K0 = first stored word, STRIDE = words per staged row. (0, 8) keeps
// the 32-byte global slot image (two b128 LDS writes); compact layouts (1, 7) / (4, 4)
// store only the words a level can still read, so more workgroups fit per CU.
template <bool ROWS, bool HALF = false, int K0 = 0, int STRIDE = EQ_WORDS>
NX_DEV uint32_t eq_stage(const EquihashDev& p, uint32_t inst, int level, int buf, uint32_t bucket, uint32_t* rows,
                         short* sid, uint32_t* bstart) {
    const uint32_t per = EQ_CAP / p.banks;
    if (threadIdx.x == 0) {
        const uint32_t* c = eq_count(p, inst, level) + (size_t)bucket * EQ_MAX_BANKS;
        uint32_t tot = 0;
        for (uint32_t k = 0; k < p.banks; ++k) {
            bstart[k] = tot;
            tot += min(c[k], per);
        }
        bstart[EQ_MAX_BANKS] = tot;
    }
    __syncthreads();
    const uint32_t n = bstart[EQ_MAX_BANKS];
    for (uint32_t i = threadIdx.x; i < n; i += EQ_BLOCK) {
        uint32_t k = 0;
        while (k + 1 < p.banks && i >= bstart[k + 1]) ++k;
        const uint32_t slot = k * per + (i - bstart[k]);
        sid[i] = (short)slot;
        if (ROWS) {
            const uint4* src = (const uint4*)(p.hashes + eq_hidx(p, buf, inst, bucket, slot));
#ifndef EQ_SEPARATE_REFS
            const uint4 lo = src[0];
            p.refs[eq_ridx(p, inst, level, bucket, slot)] = lo.x;  // bucket-contiguous: coalesced
#endif
            if constexpr (K0 == 0) {
#ifdef EQ_SEPARATE_REFS
                if (!HALF) ((uint4*)rows)[2 * i] = src[0];  // HALF: words 0..3 are never read
#else
                if (!HALF) ((uint4*)rows)[2 * i] = lo;
#endif
                ((uint4*)rows)[2 * i + 1] = src[1];
            } else {
                uint32_t w[8];
                const uint4 hi = src[1];
                w[4] = hi.x; w[5] = hi.y; w[6] = hi.z; w[7] = hi.w;
                if constexpr (K0 < 4) {
#ifdef EQ_SEPARATE_REFS
                    const uint4 lo = src[0];
#endif
                    w[1] = lo.y; w[2] = lo.z; w[3] = lo.w;
                }
#pragma unroll
                for (int k = K0; k < 8; ++k) rows[i * STRIDE + (k - K0)] = w[k];
            }
        }
    }
    __syncthreads();
    return n;
}

// Round 0: one BLAKE2b per thread -> 2 leaves -> level-0 buckets.
extern "C" __global__ __launch_bounds__(EQ_BLOCK) void eq_gen(EquihashDev p) {
    const uint32_t inst = blockIdx.y;
    const uint32_t g = blockIdx.x * EQ_BLOCK + threadIdx.x;  // digest index, < 2^20
    uint64_t m[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = p.msgs[(size_t)inst * 16 + i];
    // append le32(g) at byte offset input_len (input_len % 8 == 0 or 4 handled generically)
    {
        const uint32_t off = p.input_len;
        const uint32_t wi = off >> 3, sh = (off & 7) * 8;
        // word-aligned in practice (112 = 14*8); generic path for off % 8 == 4
        uint64_t add = (uint64_t)g << sh;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if ((uint32_t)i == wi) m[i] |= add;
        if (sh > 32) {
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if ((uint32_t)i == wi + 1) m[i] |= (uint64_t)g >> (64 - sh);
        }
    }
    uint64_t out[8];
    eq_blake2b_final(p.h0, m, (uint64_t)p.input_len + 4, out);
    // 50 digest bytes -> two 25-byte leaves, as big-endian 32-bit words
    uint8_t b[56];
#pragma unroll
    for (int i = 0; i < 7; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) b[8 * i + k] = (uint8_t)(out[i] >> (8 * k));
    }
    uint32_t* cnt = eq_count(p, inst, 0);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        uint32_t w[8];
        w[0] = 0;
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            const int base = half * 25 + 4 * i;
            const uint32_t b0 = b[base];
            const uint32_t b1 = (4 * i + 1 < 25) ? b[base + 1] : 0;
            const uint32_t b2 = (4 * i + 2 < 25) ? b[base + 2] : 0;
            const uint32_t b3 = (4 * i + 3 < 25) ? b[base + 3] : 0;
            w[i + 1] = (4 * i < 25) ? ((b0 << 24) | (b1 << 16) | (b2 << 8) | b3) : 0;
        }
        const uint32_t bucket = eq_digit<0>(w) >> 8;
        const uint32_t slot = eq_alloc_slot(p, cnt, bucket);
        if (slot < EQ_CAP) {
            uint4* dst = (uint4*)(p.hashes + eq_hidx(p, 0, inst, bucket, slot));
#ifdef EQ_SEPARATE_REFS
            dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
            p.refs[eq_ridx(p, inst, 0, bucket, slot)] = 2 * g + half;
#else
            dst[0] = make_uint4(2 * g + half, w[1], w[2], w[3]);  // word 0 carries the ref (eq_store_row)
#endif
            dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
        }
    }
}

template <int L>
NX_DEV void eq_store_row(const EquihashDev& p, uint32_t inst, uint32_t nb, uint32_t slot, const uint32_t x[8],
                         uint32_t ref) {
    uint4* dst = (uint4*)(p.hashes + eq_hidx(p, L & 1, inst, nb, slot));
#ifdef EQ_SEPARATE_REFS
    if (!eq_half_row(L)) dst[0] = make_uint4(0, x[1], x[2], x[3]);
    dst[1] = make_uint4(x[4], x[5], x[6], x[7]);
    p.refs[eq_ridx(p, inst, L, nb, slot)] = ref;
#else
    // One 32-byte write per row: word 0 (never part of the string) carries the
    // back-pointer, so row and ref share one scattered memory request. The next
    // round copies the refs of the rows it stages out to `refs` bucket by bucket,
    // i.e. as coalesced writes (profiles/r1j: the scattered write requests, not
    // bytes, bound the round kernels).
    dst[0] = make_uint4(ref, x[1], x[2], x[3]);
    dst[1] = make_uint4(x[4], x[5], x[6], x[7]);
#endif
}

// Round R (1..8): collide level R-1 on digit R-1, write level R.
// Phase 1 stages the bucket and chains rows by their 8-bit sub-digit (LDS
// atomics); each thread then walks its chain and appends every surviving pair
// to its next-level bucket (one slot atomic + one row store each).
// EQ_PAIRLIST instead lists the pairs in LDS first and emits them two per
// thread with both slot atomics in flight — measured 16 % SLOWER per solve
// (profiles/r1c_equihash), so it stays a tuning variant.
#define EQ_PAIR_MAX 992  // keeps the round's LDS under 32 KiB: 5 workgroups per CU
#ifndef EQ_EMIT_BATCH
#define EQ_EMIT_BATCH 1  // pairs whose slot atomics a thread keeps in flight together
#endif
// Compact LDS rows are the default (profiles/r1h_equihash: -4 % time per solve with the
// ref-in-slot layout); EQ_FULL_LDS restores the 32-byte staged image for A/B runs.
#ifndef EQ_FULL_LDS
#define EQ_COMPACT_LDS
#endif
#ifdef EQ_COMPACT_LDS
template <int R> constexpr int eq_lds_k0() { return eq_half_row(R - 1) ? 4 : 1; }
#else
template <int R> constexpr int eq_lds_k0() { return 0; }
#endif
// Words per staged row. Half rows (4 live words) are padded to a stride of 5 under
// EQ_LDS_PAD5 so that 64 consecutive rows hit 64 different LDS banks (stride 4: 4-way).
#ifdef EQ_LDS_PAD5
template <int R> constexpr int eq_lds_stride() { return eq_lds_k0<R>() == 4 ? 5 : (eq_lds_k0<R>() ? 8 - eq_lds_k0<R>() : EQ_WORDS); }
#else
template <int R> constexpr int eq_lds_stride() { return eq_lds_k0<R>() ? 8 - eq_lds_k0<R>() : EQ_WORDS; }
#endif

template <int R>
NX_DEV void eq_emit(const EquihashDev& p, uint32_t inst, uint32_t bucket, uint32_t* cnt, const uint32_t* rows,
                    const short* sid, const uint32_t* pr, int np) {
    constexpr int K0 = eq_lds_k0<R>(), ST = eq_lds_stride<R>();
    uint32_t slot[EQ_EMIT_BATCH], nb[EQ_EMIT_BATCH];
#pragma unroll
    for (int k = 0; k < EQ_EMIT_BATCH; ++k) {  // all slot atomics first: their latencies overlap
        if (k < np) {
            uint32_t x[8];
            eq_xor_rows<R>(rows + (pr[k] >> 16) * ST - K0, rows + (pr[k] & 0xFFFFu) * ST - K0, x);
            nb[k] = eq_digit<R>(x) >> 8;
            slot[k] = eq_alloc_slot(p, cnt, nb[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < EQ_EMIT_BATCH; ++k) {
        if (k < np && slot[k] < EQ_CAP) {
            uint32_t x[8];
            const uint32_t i = pr[k] >> 16, j = pr[k] & 0xFFFFu;
            eq_xor_rows<R>(rows + i * ST - K0, rows + j * ST - K0, x);
            eq_store_row<R>(p, inst, nb[k], slot[k], x, (bucket << 20) | ((uint32_t)sid[i] << 10) | (uint32_t)sid[j]);
        }
    }
}

// Round R (1..8): collide level R-1 on digit R-1, write level R.
// Phase 1 stages the bucket and chains rows by their 8-bit sub-digit (LDS
// atomics); each thread then walks its chain and appends every surviving pair
// to its next-level bucket (one slot atomic + one row store each), EQ_EMIT_BATCH
// pairs at a time. EQ_PAIRLIST instead lists the pairs in LDS first and emits
// them two per thread — measured 16 % SLOWER per solve (profiles/r1c_equihash).
template <int R>
NX_DEV void eq_round_impl(const EquihashDev& p) {
    constexpr int K0 = eq_lds_k0<R>(), ST = eq_lds_stride<R>();
    __shared__ __attribute__((aligned(16))) uint32_t rows[EQ_CAP * ST];
    __shared__ int head[256];
    __shared__ short nxt[EQ_CAP];
    __shared__ short sid[EQ_CAP];
    __shared__ uint32_t bstart[EQ_MAX_BANKS + 1];
#ifdef EQ_PAIRLIST
    __shared__ uint32_t pairs[EQ_PAIR_MAX];
    __shared__ uint32_t npairs;
#endif
    const uint32_t inst = blockIdx.y;
    const uint32_t bucket = blockIdx.x;
    for (int i = threadIdx.x; i < 256; i += EQ_BLOCK) head[i] = -1;
#ifdef EQ_PAIRLIST
    if (threadIdx.x == 0) npairs = 0;
#endif
    const uint32_t n = eq_stage<true, eq_half_row(R - 1), K0, ST>(p, inst, R - 1, (R - 1) & 1, bucket, rows, sid, bstart);
    for (uint32_t i = threadIdx.x; i < n; i += EQ_BLOCK) {
        const uint32_t sub = eq_digit<R - 1>(rows + i * ST - K0) & 0xFFu;
        nxt[i] = (short)atomicExch(&head[sub], (int)i);
    }
    __syncthreads();
    uint32_t* cnt = eq_count(p, inst, R);
    uint32_t pr[EQ_EMIT_BATCH];
    int np = 0;
    for (uint32_t i = threadIdx.x; i < n; i += EQ_BLOCK) {
        const uint32_t* a = rows + i * ST - K0;
        int j = nxt[i];
        for (int steps = 0; j >= 0 && steps < EQ_MAX_CHAIN; j = nxt[j], ++steps) {
            uint32_t x[8];
            eq_xor_rows<R>(a, rows + (uint32_t)j * ST - K0, x);
            if (eq_zero_from<R>(x)) continue;  // identical remainder -> only duplicate indices
#ifdef EQ_PAIRLIST
            const uint32_t k = atomicAdd(&npairs, 1u);
            if (k < EQ_PAIR_MAX) {
                pairs[k] = (i << 16) | (uint32_t)j;
                continue;
            }
#endif
            pr[np++] = (i << 16) | (uint32_t)j;
            if (np == EQ_EMIT_BATCH) {
                eq_emit<R>(p, inst, bucket, cnt, rows, sid, pr, np);
                np = 0;
            }
        }
    }
    if (np) eq_emit<R>(p, inst, bucket, cnt, rows, sid, pr, np);
#ifdef EQ_PAIRLIST
    __syncthreads();
    const uint32_t npl = min(npairs, (uint32_t)EQ_PAIR_MAX);
    for (uint32_t k = threadIdx.x; k < npl; k += 2 * EQ_BLOCK) {
        uint32_t pp[2] = {pairs[k], k + EQ_BLOCK < npl ? pairs[k + EQ_BLOCK] : 0u};
        for (int q = 0; q < (k + EQ_BLOCK < npl ? 2 : 1); ++q) eq_emit<R>(p, inst, bucket, cnt, rows, sid, &pp[q], 1);
    }
#endif
}

#define EQ_ROUND_KERNEL(R) \
    extern "C" __global__ __launch_bounds__(EQ_BLOCK) void eq_round##R(EquihashDev p) { eq_round_impl<R>(p); }
EQ_ROUND_KERNEL(1)
EQ_ROUND_KERNEL(2)
EQ_ROUND_KERNEL(3)
EQ_ROUND_KERNEL(4)
EQ_ROUND_KERNEL(5)
EQ_ROUND_KERNEL(6)
EQ_ROUND_KERNEL(7)
EQ_ROUND_KERNEL(8)

// Final round: level-8 rows colliding on d_8 and d_9 (40 bits) are candidates.
extern "C" __global__ __launch_bounds__(EQ_BLOCK) void eq_final(EquihashDev p) {
    __shared__ uint32_t d9[EQ_CAP];
    __shared__ int head[256];
    __shared__ short nxt[EQ_CAP];
    __shared__ short sid[EQ_CAP];
    __shared__ uint32_t bstart[EQ_MAX_BANKS + 1];
    const uint32_t inst = blockIdx.y;
    const uint32_t bucket = blockIdx.x;
    for (int i = threadIdx.x; i < 256; i += EQ_BLOCK) head[i] = -1;
    const uint32_t n = eq_stage<false>(p, inst, 8, 0, bucket, nullptr, sid, bstart);
    for (uint32_t i = threadIdx.x; i < n; i += EQ_BLOCK) {
        // level 8 lives in buffer 8 & 1 = 0
        const uint32_t* w = p.hashes + eq_hidx(p, 0, inst, bucket, (uint32_t)sid[i]);
#ifndef EQ_SEPARATE_REFS
        p.refs[eq_ridx(p, inst, 8, bucket, (uint32_t)sid[i])] = w[0];
#endif
        const uint32_t d8 = eq_digit<8>(w), dd = eq_digit<9>(w);
        d9[i] = dd;
        nxt[i] = (short)atomicExch(&head[d8 & 0xFFu], (int)i);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += EQ_BLOCK) {
        for (int j = nxt[i], steps = 0; j >= 0 && steps < EQ_MAX_CHAIN; j = nxt[j], ++steps) {
            if (d9[i] != d9[(uint32_t)j]) continue;
            uint32_t* c = p.cands + (size_t)inst * (1 + 2 * EQ_MAX_CAND);
            const uint32_t k = atomicAdd(&c[0], 1u);
            if (k < EQ_MAX_CAND) {
                c[1 + 2 * k] = bucket * EQ_CAP + (uint32_t)sid[i];
                c[2 + 2 * k] = bucket * EQ_CAP + (uint32_t)sid[j];
            }
        }
    }
}

// Reconstruct the 512 leaf indices of every candidate (equihash_device.hpp eq_reconstruct_body).
extern "C" __global__ __launch_bounds__(EQ_BLOCK) void eq_reconstruct(EquihashDev p) {
    const uint32_t inst = blockIdx.y;
    eq_reconstruct_body<EQ_CAP, EQ_BLOCK>(p.refs + (size_t)inst * EQ_LEVELS * EQ_BUCKETS * EQ_CAP,
                                          p.cands + (size_t)inst * (1 + 2 * EQ_MAX_CAND),
                                          p.sols + (size_t)inst * (1 + EQ_MAX_SOL * 512));
}

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
