// Equihash(200,9) Wagner solver for gfx950 with private slot segments (new; the reference has
// no Equihash — SURVEY §0.4 / Appendix D). CPU golden model: csrc/pow/equihash.cpp.
//
// Why a second solver. The global-slot solver (equihash.hip) appends every output row with a
// returning global atomicAdd on its bucket's counter, and its 4096 one-bucket workgroups per
// round each pay that round trip before their stores. Measured on MI355X (profiles/README r2d):
// removing the atomics alone changed nothing (the rounds are bound by the scattered row stores,
// two 16-byte requests per row), so this engine also (1) packs rows into ONE 16-byte store from
// level 5 on (eq_pack16) and (2) pipelines each workgroup's bucket sequence so that the gathers
// of the next bucket run beside the collisions of the current one. Device time per 8-solve
// batch: 5.64 ms against 6.54 ms for the global-slot engine.
//
// Here nothing per row is global. A round runs P = p.groups workgroups per instance; workgroup
// w processes the source buckets b ≡ w (mod P) one after another, and owns, in EVERY bucket of
// the level it writes, a private segment of C = p.seg row slots (P * C = EQP_SLOTS). Its slot
// counters (4096 buckets, packed u16 pairs) live in LDS, so appending a row is one LDS atomic
// and fire-and-forget stores. When the workgroup is done it writes its 4096 counts
// (clamped to C) as one coalesced 4 KiB row of `counts`.
//
// The next round stages bucket b by reading the P counts of b (one byte from each writer's row;
// the whole level's counts are 512 KiB and stay in L2 / the Infinity Cache), prefix-summing them
// in one wave, and gathering each segment's rows, which are contiguous. Staged rows get a
// compact index (< EQP_STAGE); the round copies their back-pointers out to
// refs[level][b][index], so a back-pointer (bucket << 20 | index a << 10 | index b) fits in 32
// bits and reconstruction (equihash_device.hpp) is the same as for the global-slot solver.
//
// Layouts (num_inst = ni):
//   hashes [2][ni][BUCKETS][EQP_SLOTS][8] u32  (levels alternate between the two buffers)
//   counts [ni][LEVELS][P][BUCKETS] u8
//   refs   [ni][LEVELS][BUCKETS][EQP_REF_STRIDE] u32
// Overflowing segments or staging areas drop rows (counted in p.stats per level), and a chain of
// equal sub-digits longer than EQ_MAX_CHAIN is cut (counted in p.stats[EQP_STAT_CHAIN]); at
// C = 32 for a mean of 8 rows per segment, 768 staged for a mean of 512 per bucket and 24 for a
// mean chain of 2, none of them has been seen in any run. The host (ops/equihash.py) re-solves an
// instance with any such count on the golden solver, so the solution set is exact either way.
#include "equihash_device.hpp"

#define EQP_BLOCK 512

// Word offset of a row slot of `level` (buffer level & 1): 32-byte slots, 16-byte slots for the
// packed levels (so a segment's rows stay contiguous).
NX_DEV size_t eqp_hidx(const EquihashPsDev& p, int level, uint32_t inst, uint32_t bucket, uint32_t grp, uint32_t slot) {
    const size_t buf_words = (size_t)p.num_inst * EQ_BUCKETS * EQP_SLOTS * EQ_WORDS;  // one level buffer
    const size_t row = ((size_t)inst * EQ_BUCKETS + bucket) * EQP_SLOTS + grp * p.seg + slot;
    return (size_t)(level & 1) * buf_words + row * (eq_half_row(level) ? 4 : EQ_WORDS);
}

// LDS slot counters, two u16 per word (the counts of one workgroup never reach 2^16).
NX_DEV uint32_t eqp_take_slot(uint32_t* cnt2, uint32_t nb) {
    const uint32_t sh = (nb & 1u) << 4;
    return (atomicAdd(&cnt2[nb >> 1], 1u << sh) >> sh) & 0xFFFFu;
}

NX_DEV void eqp_clear_counts(uint32_t* cnt2) {
    for (uint32_t k = threadIdx.x; k < EQ_BUCKETS / 2; k += EQP_BLOCK) cnt2[k] = 0;
}

// This workgroup's 4096 segment fills of `level`, clamped to C, as one coalesced u8 row.
// `dropped` (this thread's staging overflow) plus the segment overflow go to p.stats.
NX_DEV void eqp_flush_counts(const EquihashPsDev& p, uint32_t inst, int level, const uint32_t* cnt2,
                             uint32_t dropped) {
    uint32_t* out = (uint32_t*)(p.counts + (((size_t)inst * EQ_LEVELS + level) * p.groups + blockIdx.x) * EQ_BUCKETS);
    for (uint32_t k = threadIdx.x; k < EQ_BUCKETS / 4; k += EQP_BLOCK) {
        const uint32_t a = cnt2[2 * k], b = cnt2[2 * k + 1];
        const uint32_t c[4] = {a & 0xFFFFu, a >> 16, b & 0xFFFFu, b >> 16};
        uint32_t packed = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t v = min(c[q], p.seg);
            dropped += c[q] - v;
            packed |= v << (8 * q);
        }
        out[k] = packed;
    }
    if (dropped) atomicAdd(&p.stats[inst * EQP_STATS + level], dropped);
}

// Round 0: BLAKE2b of this workgroup's 2^20 / P digest indices, 2 leaves each, appended to
// this workgroup's segment of their level-0 bucket (word 0 = leaf index).
extern "C" __global__ __launch_bounds__(EQP_BLOCK) void eqp_gen(EquihashPsDev p) {
    __shared__ uint32_t cnt2[EQ_BUCKETS / 2];
    const uint32_t inst = blockIdx.y, grp = blockIdx.x;
    eqp_clear_counts(cnt2);
    __syncthreads();
    const uint32_t per = (1u << 20) / p.groups;
    const uint64_t* msg = p.msgs + (size_t)inst * 16;
    for (uint32_t t = threadIdx.x; t < per; t += EQP_BLOCK) {
        const uint32_t g = grp * per + t;
        uint64_t out[8];
        eq_digest(msg, p.h0, p.input_len, g, out);
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            uint32_t w[8];
            eq_leaf_words(out, half, w);
            const uint32_t nb = eq_digit<0>(w) >> 8;
            const uint32_t slot = eqp_take_slot(cnt2, nb);
            if (slot < p.seg) {
                uint4* dst = (uint4*)(p.hashes + eqp_hidx(p, 0, inst, nb, grp, slot));
                dst[0] = make_uint4(2 * g + half, w[1], w[2], w[3]);
                dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
            }
        }
    }
    __syncthreads();
    eqp_flush_counts(p, inst, 0, cnt2, 0);
}

// Counts of bucket b of `level` into lane registers of the calling wave (lane l holds the counts
// of segments l*per .. l*per+per-1, per = P / 64 rounded up).
NX_DEV void eqp_load_counts(const EquihashPsDev& p, uint32_t inst, int level, uint32_t b, uint32_t v[4]) {
    const uint32_t P = p.groups, lane = threadIdx.x & 63, per = (P + 63) / 64;
    const uint8_t* cin = p.counts + ((size_t)inst * EQ_LEVELS + level) * P * EQ_BUCKETS + b;
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t g = lane * per + q;
        v[q] = (q < per && g < P) ? (uint32_t)cin[(size_t)g * EQ_BUCKETS] : 0u;
    }
}

// Wave-wide exclusive prefix of the counts held by eqp_load_counts into segc; returns the total.
NX_DEV uint32_t eqp_wave_scan(uint32_t P, const uint32_t v[4], uint32_t* segc) {
    const uint32_t lane = threadIdx.x & 63, per = (P + 63) / 64;
    const uint32_t s = v[0] + v[1] + v[2] + v[3];
    uint32_t x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if ((int)lane >= o) x += y;
    }
    uint32_t run = x - s;
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t g = lane * per + q;
        if (q < per && g < P) segc[g] = run;
        run += v[q];
    }
    __builtin_amdgcn_wave_barrier();
    return __shfl(x, 63, 64);
}

// Producer threads pt = 0..NP-1 gather the staged rows pos = pt, pt + NP, ... of bucket b of
// `level` into LDS rows (words K0..7 at stride ST) and copy their back-pointers to
// refs[level][b][pos]. A row's segment is found by binary search over the prefix segc, so every
// load is a real row (about 4 per producer lane per bucket, all in flight together).
template <int K0, int ST, uint32_t NP>
NX_DEV void eqp_gather_rows(const EquihashPsDev& p, uint32_t inst, int level, uint32_t b, const uint32_t* segc,
                            uint32_t n, uint32_t* rows, uint32_t pt) {
    constexpr int BATCH = 4;
    const bool packed = eq_half_row(level);
    const uint32_t P = p.groups;
    uint32_t* refs = p.refs + (((size_t)inst * EQ_LEVELS + level) * EQ_BUCKETS + b) * EQP_REF_STRIDE;
#pragma unroll 1
    for (uint32_t p0 = pt; p0 < n; p0 += NP * BATCH) {
        uint4 lo[BATCH], hi[BATCH];
#pragma unroll
        for (int k = 0; k < BATCH; ++k) {
            const uint32_t pos = p0 + k * NP;
            if (pos >= n) continue;
            uint32_t a = 0, z = P;  // largest segment whose prefix is <= pos
            while (z - a > 1) {
                const uint32_t mid = (a + z) >> 1;
                if (segc[mid] <= pos) a = mid; else z = mid;
            }
            const uint4* src = (const uint4*)(p.hashes + eqp_hidx(p, level, inst, b, a, pos - segc[a]));
            lo[k] = src[0];
            if (!packed) hi[k] = src[1];
        }
#pragma unroll
        for (int k = 0; k < BATCH; ++k) {
            const uint32_t pos = p0 + k * NP;
            if (pos >= n) continue;
            uint32_t w[8];
            if (packed) {
                eq_unpack16(lo[k], level == 5 ? b << 16 : 0u, w);
            } else {
                w[1] = lo[k].y; w[2] = lo[k].z; w[3] = lo[k].w;
                w[4] = hi[k].x; w[5] = hi[k].y; w[6] = hi[k].z; w[7] = hi[k].w;
            }
            refs[pos] = lo[k].x;
#pragma unroll
            for (int q = K0; q < 8; ++q) rows[pos * ST + (q - K0)] = w[q];
        }
    }
}

// Round R (1..8): collide level R-1 on digit R-1 bucket by bucket, write level R. R = 9 is the
// final round: level-8 rows colliding on d_8 and d_9 (40 bits) become candidates.
//
// Producer / consumer split: waves 0-1 stage the NEXT bucket (count scan, row gathers into the
// other LDS row buffer, back-pointer copies, the counts of the bucket after that) while waves
// 2..7 chain and collide the current bucket and emit rows. A wave's vmcnt counts its loads and
// stores together in issue order, so keeping the gathers out of the emitting waves means no load
// ever waits behind a scattered row store; the gathers' latency hides behind the collisions.
// Two barriers per bucket: after staging (A: rows ready) and after chaining (B: links ready).
template <int R>
NX_DEV void eqp_round_impl(const EquihashPsDev& p) {
    constexpr int K0 = eq_half_row(R - 1) ? 4 : 1;  // first word a level-(R-1) row still needs
    constexpr int ST = 8 - K0;
    constexpr uint32_t NP = 128, NC = EQP_BLOCK - NP;  // producer / consumer threads
    __shared__ uint32_t cnt2[EQ_BUCKETS / 2];
    __shared__ __attribute__((aligned(16))) uint32_t rows[2][EQP_STAGE * ST];
    __shared__ int head[256];
    __shared__ short nxt[EQP_STAGE];
    __shared__ uint32_t segc[NP / 64][256];  // one prefix copy per producer wave (no cross-wave sync)
    __shared__ uint32_t nstaged[2];
    // P = writers per level (the counts layout); the workgroups stride over the buckets by the
    // grid width, which is P for rounds 1..8 (workgroup = writer) and wider for the final round
    const uint32_t inst = blockIdx.y, grp = blockIdx.x, P = p.groups, G = gridDim.x;
    const bool producer = threadIdx.x < NP;
    const uint32_t ct = threadIdx.x - NP;
    uint32_t* my_segc = segc[threadIdx.x / 64 % (NP / 64)];
    eqp_clear_counts(cnt2);
    for (uint32_t i = threadIdx.x; i < 256; i += EQP_BLOCK) head[i] = -1;
    uint32_t cv[4] = {0, 0, 0, 0};
    uint32_t dropped = 0, truncated = 0, staged_max = 0;
    // every producer wave scans the counts itself and gathers rows pos = thread, thread + NP, ...
    auto stage = [&](uint32_t bk, uint32_t buf) {
        const uint32_t total = eqp_wave_scan(P, cv, my_segc);
        const uint32_t n = min(total, (uint32_t)EQP_STAGE);
        eqp_gather_rows<K0, ST, NP>(p, inst, R - 1, bk, my_segc, n, rows[buf], threadIdx.x);
        if (threadIdx.x == 0) {
            nstaged[buf] = n;
            dropped += total - n;
            staged_max = max(staged_max, total);
        }
        if (bk + G < EQ_BUCKETS) eqp_load_counts(p, inst, R - 1, bk + G, cv);
    };
    if (producer) {  // prologue: stage the first bucket, prefetch the counts of the second
        eqp_load_counts(p, inst, R - 1, grp, cv);
        stage(grp, 0);
    }
    uint32_t cur = 0;
    for (uint32_t b = grp; b < EQ_BUCKETS; b += G, cur ^= 1) {
        __syncthreads();  // A: rows[cur] staged, head reset, previous bucket's emission done
        const uint32_t n = nstaged[cur];
        const uint32_t* rc = rows[cur];
        if (!producer) {
            for (uint32_t i = ct; i < n; i += NC) {
                const uint32_t sub = eq_digit<R - 1>(rc + i * ST - K0) & 0xFFu;
                nxt[i] = (short)atomicExch(&head[sub], (int)i);
            }
        }
        __syncthreads();  // B: chain links of the current bucket complete
        if (producer) {
            for (uint32_t i = threadIdx.x; i < 256; i += NP) head[i] = -1;  // chain building is over
            if (b + G < EQ_BUCKETS) stage(b + G, cur ^ 1);
        } else {
            for (uint32_t i = ct; i < n; i += NC) {
                const uint32_t* a = rc + i * ST - K0;
                if constexpr (R == 9) {  // final round: equal d_8 (chain) and d_9 make a candidate
                    const uint32_t di = eq_digit<9>(a);
                    int j = nxt[i], steps = 0;
                    for (; j >= 0 && steps < EQ_MAX_CHAIN; j = nxt[j], ++steps) {
                        if (di != eq_digit<9>(rc + (uint32_t)j * ST - K0)) continue;
                        uint32_t* c = p.cands + (size_t)inst * (1 + 2 * EQ_MAX_CAND);
                        const uint32_t k = atomicAdd(&c[0], 1u);
                        if (k < EQ_MAX_CAND) {
                            c[1 + 2 * k] = b * EQP_REF_STRIDE + i;
                            c[2 + 2 * k] = b * EQP_REF_STRIDE + (uint32_t)j;
                        }
                    }
                    truncated += j >= 0;  // the chain went on past EQ_MAX_CHAIN: pairs not tried
                    continue;
                }
                int j = nxt[i], steps = 0;
                for (; j >= 0 && steps < EQ_MAX_CHAIN; j = nxt[j], ++steps) {
                    uint32_t x[8];
                    eq_xor_rows<R>(a, rc + (uint32_t)j * ST - K0, x);
                    if (eq_zero_from<R>(x)) continue;  // identical remainder: only duplicate indices
                    const uint32_t nb = eq_digit<R>(x) >> 8;
                    const uint32_t slot = eqp_take_slot(cnt2, nb);
                    if (slot < p.seg) {
                        uint4* dst = (uint4*)(p.hashes + eqp_hidx(p, R, inst, nb, grp, slot));
                        const uint32_t ref = (b << 20) | (i << 10) | (uint32_t)j;
                        if constexpr (eq_half_row(R)) {
                            dst[0] = eq_pack16(ref, x);
                        } else {
                            dst[0] = make_uint4(ref, x[1], x[2], x[3]);
                            dst[1] = make_uint4(x[4], x[5], x[6], x[7]);
                        }
                    }
                }
                truncated += j >= 0;
            }
        }
    }
    __syncthreads();
    // staging overflow (rows of a level-(R-1) bucket beyond EQP_STAGE) and segment overflow (level R
    // rows beyond a segment) are counted apart
    if (dropped) atomicAdd(&p.stats[inst * EQP_STATS + EQP_STAT_STAGE], dropped);
    if (threadIdx.x == 0) atomicMax(&p.stats[inst * EQP_STATS + EQP_STAT_STAGE_MAX], staged_max);
    if constexpr (R < 9) eqp_flush_counts(p, inst, R, cnt2, 0);
    if (truncated) atomicAdd(&p.stats[inst * EQP_STATS + EQP_STAT_CHAIN], truncated);
}

// 2 workgroups of 512 per CU (4 waves per SIMD): at most 128 VGPRs.
#define EQP_ROUND_KERNEL(R) \
    extern "C" __global__ __launch_bounds__(EQP_BLOCK, 4) void eqp_round##R(EquihashPsDev p) { eqp_round_impl<R>(p); }
EQP_ROUND_KERNEL(1)
EQP_ROUND_KERNEL(2)
EQP_ROUND_KERNEL(3)
EQP_ROUND_KERNEL(4)
EQP_ROUND_KERNEL(5)
EQP_ROUND_KERNEL(6)
EQP_ROUND_KERNEL(7)
EQP_ROUND_KERNEL(8)

extern "C" __global__ __launch_bounds__(EQP_BLOCK, 4) void eqp_final(EquihashPsDev p) { eqp_round_impl<9>(p); }

// Leaf indices of every candidate (shared body: equihash_device.hpp).
extern "C" __global__ __launch_bounds__(256) void eqp_reconstruct(EquihashPsDev p) {
    const uint32_t inst = blockIdx.y;
    eq_reconstruct_body<EQP_REF_STRIDE, 256>(p.refs + (size_t)inst * EQ_LEVELS * EQ_BUCKETS * EQP_REF_STRIDE,
                                             p.cands + (size_t)inst * (1 + 2 * EQ_MAX_CAND),
                                             p.sols + (size_t)inst * (1 + EQ_MAX_SOL * 512));
}
