// Equihash(200,9) Wagner solver for gfx950 with coarse destination buckets (new; the reference has
// no Equihash — SURVEY §0.4 / Appendix D). CPU golden model: csrc/pow/equihash.cpp.
//
// What bounds a Wagner round on MI355X is its scattered row stores: every round appends 2^21
// rows per instance to random buckets, and at 4096 buckets per level each row leaves the L2 as
// its own partial-line write (1.06-1.18 EA write requests per row, profiles/README r4r/r4l).
// The private-slot solver (equihash_ps.hip) sits on that floor. This solver keeps fewer lines
// open instead: a level's rows are stored by the top EQC_COARSE_BITS (8) bits of the digit they
// collide on next, so a writer appends to 256 segments instead of 4096 and the L2 merges its
// appends into lines before they go out. The store probe (tools/eq_runs_probe.hip, profiles r5a)
// in the solver's shape: 0.43-0.54 requests and 0.32-0.44 ms per 33.5M rows at 256 buckets against
// 1.06-1.18 and 0.71-0.87 ms at 4096.
//
// The collisions still need the full 20-bit digit. A round's work item is a fine bucket = (coarse
// bucket, slice): the next EQC_SLICE_BITS (2) digit bits, carried in the row. The workgroup that
// owns a coarse bucket processes its 4 slices back to back and reads the coarse bucket once per
// slice, keeping the slice's rows (~2048; the probe: re-reads of a bucket right after the first
// pass hit the L2). Within a fine bucket rows chain on the remaining 10 digit bits (LDS linked
// lists, as the private-slot solver's 8-bit sub-digits).
//
// Back-pointers: a fine bucket of ~2048 staged rows needs 12-bit indices, and (bucket, index a,
// index b) no longer fits 32 bits. So every emitted row gets an id (its writer x pmax + the
// writer's emission count, one wave-aggregated LDS atomic), stored as the row's word 0, and the
// ids of its two parent rows go to a pair log: pairs[level][id] = (parent a, parent b), written
// coalesced (consecutive ids per wave). Level-0 ids are leaf indices, so reconstruction walks
// pairs[8] .. pairs[1] from a candidate's two level-8 ids straight to its 512 leaves.
//
// Row format (level L): word 0 = id, then the row's bits [20L + 8, 200) big-endian and contiguous
// (the payload: slice bits [0, 2), chain key [2, 12), next digit's coarse bits [12, 20), ...).
// Bits [20L, 20L + 8) are the coarse bucket and live in the row's address. Payload words 6, 6, 5,
// 5, 4, 3, 3, 2, 1 for levels 0..8; rows are stored unpadded (id + payload).
//
// Layouts (num_inst = ni, P writers per instance, seg rows per segment: mean 2^13 / P + 8 sigma):
//   hashes [2][ni][COARSE][P][seg][words(level)]  (levels alternate between two buffers)
//   counts [ni][LEVELS][P][COARSE] u16
//   pairs  [ni][LEVELS][P * pmax][2]
// Every device-side cap (segment slots, staged rows, chain length, candidates, pair ids) is
// counted in p.stats; the host re-solves an instance with any count on the golden solver, so the
// solution set is exact either way (ops/equihash.py).
#include "equihash_device.hpp"

#ifndef EQC_BLOCK
#define EQC_BLOCK 1024  // threads per workgroup (the launcher's `block`)
#endif
#ifndef EQC_MIN_WAVES
#define EQC_MIN_WAVES 4  // waves per SIMD the round kernels are register-limited for (4: 128 VGPRs)
#endif
#ifndef EQC_NP
#define EQC_NP 448  // producer threads of a round workgroup (7 of its 16 waves)
#endif
#ifndef EQC_BATCH
#define EQC_BATCH 6  // rows in flight per producer lane while a coarse bucket streams in
#endif

constexpr uint32_t CB = EQC_COARSE_BITS, SB = EQC_SLICE_BITS, KB = 20 - CB - SB;
constexpr uint32_t NCO = EQC_COARSE, NSL = 1u << SB, NKEY = 1u << KB;
static_assert(KB >= 6 && KB <= 12, "chain key width");

// The slice of a row (payload bits [0, SB)); every row is in slice 0 without slices.
NX_DEV uint32_t eqc_slice(uint32_t w1) {
    if constexpr (SB == 0) return 0;
    else return w1 >> (32 - SB);
}

// Payload words of a level-L row (bits [20L + CB, 200)).
constexpr int eqc_payload(int level) { return (200 - 20 * level - (int)CB + 31) / 32; }
constexpr int eqc_words(int level) { return 1 + eqc_payload(level); }
// LDS words per staged row: a 3-word payload is padded to 4 (one ds_read_b128 per row).
constexpr int eqc_lds_stride(int level) { return eqc_payload(level) == 3 ? 4 : eqc_payload(level); }
static_assert(eqc_words(0) <= EQC_ROW_WORDS, "row buffer width");

template <int N>
struct __attribute__((aligned(4))) EqcRow {
    uint32_t w[N];
};

// Row slot of level L: a (coarse bucket, writer) segment's rows are contiguous.
template <int L>
NX_DEV uint32_t* eqc_row(const EquihashCbDev& p, uint32_t inst, uint32_t d, uint32_t w, uint32_t slot) {
    const size_t buf_words = (size_t)p.num_inst * NCO * p.groups * p.seg * EQC_ROW_WORDS;  // one level buffer
    const size_t row = (((size_t)inst * NCO + d) * p.groups + w) * p.seg + slot;
    return p.hashes + (size_t)(L & 1) * buf_words + row * eqc_words(L);
}

NX_DEV uint32_t eqc_lane() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// Wave-aggregated allocation on an LDS counter: one atomic per wave for its active lanes, which
// get consecutive values in lane order.
NX_DEV uint32_t eqc_wave_alloc(uint32_t* ctr) {
    const uint64_t m = __ballot(1);
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (eqc_lane() == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader, 64);
    return base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

NX_DEV void eqc_clear(uint32_t* cnt) {
    for (uint32_t k = threadIdx.x; k < NCO; k += EQC_BLOCK) cnt[k] = 0;
}

// This workgroup's segment fills of `level` (clamped to seg) as one coalesced u16 row; the
// overflow goes to p.stats[level].
NX_DEV void eqc_flush_counts(const EquihashCbDev& p, uint32_t inst, uint32_t grp, int level, const uint32_t* cnt) {
    uint16_t* out = p.counts + (((size_t)inst * EQ_LEVELS + level) * p.groups + grp) * NCO;
    uint32_t dropped = 0;
    for (uint32_t k = threadIdx.x; k < NCO; k += EQC_BLOCK) {
        const uint32_t v = min(cnt[k], p.seg);
        dropped += cnt[k] - v;
        out[k] = (uint16_t)v;
    }
    if (dropped) atomicAdd(&p.stats[inst * EQP_STATS + level], dropped);
}

// Round 0: BLAKE2b of this workgroup's 2^20 / P digest indices, 2 leaves each, appended to this
// workgroup's segment of their coarse bucket (word 0 = the leaf index = the level-0 id).
extern "C" __global__ __launch_bounds__(EQC_BLOCK) void eqc_gen(EquihashCbDev p) {
    __shared__ uint32_t cnt[NCO];
    if (p.coarse != NCO) return;  // a code object of another geometry than the host sized: no rows
    const uint32_t inst = blockIdx.y, grp = blockIdx.x;
    eqc_clear(cnt);
    __syncthreads();
    const uint32_t per = (1u << 20) / p.groups;
    const uint64_t* msg = p.msgs + (size_t)inst * 16;
    for (uint32_t t = threadIdx.x; t < per; t += EQC_BLOCK) {
        const uint32_t g = grp * per + t;
        uint64_t out[8];
        eq_digest(msg, p.h0, p.input_len, g, out);
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            uint32_t w[8];
            eq_leaf_words(out, half, w);
            const uint32_t nb = w[1] >> (32 - CB);  // leaf bits [0, CB)
            const uint32_t slot = atomicAdd(&cnt[nb], 1u);
            if (slot < p.seg) {
                EqcRow<eqc_words(0)> r;
                r.w[0] = 2 * g + half;
#pragma unroll
                for (int k = 0; k < eqc_payload(0); ++k)
                    r.w[1 + k] = (w[k + 1] << CB) | (k + 2 <= 7 ? w[k + 2] >> (32 - CB) : 0u);
                *(EqcRow<eqc_words(0)>*)eqc_row<0>(p, inst, nb, grp, slot) = r;
            }
        }
    }
    __syncthreads();
    eqc_flush_counts(p, inst, grp, 0, cnt);
}

// Counts of coarse bucket d of `level` into the lane registers of the calling wave (lane l holds
// the counts of writers l*per .. l*per+per-1, per = P / 64 rounded up).
NX_DEV void eqc_load_counts(const EquihashCbDev& p, uint32_t inst, int level, uint32_t d, uint32_t v[4]) {
    const uint32_t P = p.groups, lane = eqc_lane(), per = (P + 63) / 64;
    const uint16_t* cin = p.counts + ((size_t)inst * EQ_LEVELS + level) * P * NCO + d;
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t g = lane * per + q;
        v[q] = (q < per && g < P) ? (uint32_t)cin[(size_t)g * NCO] : 0u;
    }
}

// Wave-wide exclusive prefix of the counts held by eqc_load_counts into segc; returns the total.
NX_DEV uint32_t eqc_wave_scan(uint32_t P, const uint32_t v[4], uint32_t* segc) {
    const uint32_t lane = eqc_lane(), per = (P + 63) / 64;
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

// Producer threads stage slice `s` of coarse bucket d of level L: every row of the bucket (its P
// segments as one list of `total` rows; a row's segment by binary search over the prefix segc) is
// read, and the rows of the slice are appended to the LDS buffer (payload at stride ST, ids apart)
// at positions from a wave-aggregated counter. Returns the rows this lane dropped at the cap.
template <int L, uint32_t NP>
NX_DEV uint32_t eqc_stage_slice(const EquihashCbDev& p, uint32_t inst, uint32_t d, uint32_t s, const uint32_t* segc,
                                uint32_t total, uint32_t* rows, uint32_t* ids, uint32_t* nstaged) {
    constexpr int BATCH = EQC_BATCH, W = eqc_words(L), PL = eqc_payload(L), ST = eqc_lds_stride(L);
    const uint32_t P = p.groups, pt = threadIdx.x, wave0 = pt & ~63u;
    uint32_t dropped = 0;
#pragma unroll 1
    for (uint32_t p0 = wave0; p0 < total; p0 += NP * BATCH) {  // wave-uniform loop
        EqcRow<W> r[BATCH];
        bool valid[BATCH];
#pragma unroll
        for (int k = 0; k < BATCH; ++k) {
            const uint32_t pos = p0 + (pt - wave0) + k * NP;
            valid[k] = pos < total;
            if (!valid[k]) continue;
            uint32_t a = 0, z = P;  // largest segment whose prefix is <= pos
            while (z - a > 1) {
                const uint32_t mid = (a + z) >> 1;
                if (segc[mid] <= pos) a = mid; else z = mid;
            }
            r[k] = *(const EqcRow<W>*)eqc_row<L>(p, inst, d, a, pos - segc[a]);
        }
#pragma unroll
        for (int k = 0; k < BATCH; ++k) {
            const bool keep = valid[k] && eqc_slice(r[k].w[1]) == s;
            if (__ballot(keep) == 0) continue;  // wave-uniform
            if (!keep) continue;
            const uint32_t idx = eqc_wave_alloc(nstaged);
            if (idx >= EQC_STAGE) {
                ++dropped;
                continue;
            }
            ids[idx] = r[k].w[0];
#pragma unroll
            for (int q = 0; q < ST; ++q) rows[idx * ST + q] = q < PL ? r[k].w[1 + q] : 0u;
        }
    }
    return dropped;
}

// Round R (1..8): collide level R-1 on digit R-1 fine bucket by fine bucket, write level R.
// R = 9 is the final round: level-8 rows equal on d_8 and d_9 (40 bits) become candidates.
//
// Producer / consumer split as in the private-slot solver: the first EQC_NP threads (7 waves)
// stage the NEXT fine bucket (a coarse bucket's counts scan, its rows streamed, the slice kept)
// while the other 9 waves chain and collide the current one and emit rows. Two barriers per fine
// bucket: after staging (A: rows ready) and after chaining (B: links ready).
template <int R>
NX_DEV void eqc_round_impl(const EquihashCbDev& p) {
    constexpr int ST = eqc_lds_stride(R - 1);  // LDS words per staged level-(R-1) row
    constexpr uint32_t NP = EQC_NP, NC = EQC_BLOCK - NP;
    __shared__ uint32_t cnt[NCO];
    __shared__ __attribute__((aligned(16))) uint32_t rows[2][EQC_STAGE * ST];
    __shared__ uint32_t ids[2][EQC_STAGE];
    __shared__ int head[NKEY];
    __shared__ short nxt[EQC_STAGE];
    __shared__ uint32_t segc[NP / 64][EQC_MAX_P];  // one prefix copy per producer wave
    __shared__ uint32_t nstaged[2];
    __shared__ uint32_t pcount;
    if (p.coarse != NCO) return;  // geometry mismatch (whole workgroup): nothing staged or emitted
    const uint32_t inst = blockIdx.y, grp = blockIdx.x;
    const uint32_t P = p.groups, G = gridDim.x;
    const bool producer = threadIdx.x < NP;
    const uint32_t ct = threadIdx.x - NP;
    uint32_t* my_segc = segc[threadIdx.x / 64 % (NP / 64)];
    eqc_clear(cnt);
    for (uint32_t i = threadIdx.x; i < NKEY; i += EQC_BLOCK) head[i] = -1;
    if (threadIdx.x == 0) {
        nstaged[0] = nstaged[1] = 0;
        pcount = 0;
    }
    __syncthreads();
    // work item k of this workgroup: coarse bucket grp + G * (k / NSL), slice k % NSL (the slices
    // of a coarse bucket back to back, so its re-reads find it in the L2)
    const uint32_t items = grp < NCO ? ((NCO - 1 - grp) / G + 1) * NSL : 0;
    auto coarse = [&](uint32_t k) { return grp + G * (k / NSL); };
    uint32_t cv[4] = {0, 0, 0, 0};
    uint32_t total = 0;  // rows of the coarse bucket being staged (producer waves, after the scan)
    uint32_t dropped = 0, truncated = 0, staged_max = 0, lost_ids = 0;
    auto stage = [&](uint32_t k, uint32_t buf) {
        const uint32_t d = coarse(k), s = k % NSL;
        if (s == 0) total = eqc_wave_scan(P, cv, my_segc);  // counts loaded one item ahead
        dropped += eqc_stage_slice<R - 1, NP>(p, inst, d, s, my_segc, total, rows[buf], ids[buf], &nstaged[buf]);
        if (s == NSL - 1 && k + 1 < items) eqc_load_counts(p, inst, R - 1, coarse(k + 1), cv);
    };
    if (producer && items) {  // prologue: stage the first item
        eqc_load_counts(p, inst, R - 1, coarse(0), cv);
        stage(0, 0);
    }
    uint32_t cur = 0;
    for (uint32_t k = 0; k < items; ++k, cur ^= 1) {
        __syncthreads();  // A: rows[cur] staged, head reset, previous item's emission done
        const uint32_t got = nstaged[cur];
        const uint32_t n = min(got, (uint32_t)EQC_STAGE);
        const uint32_t* rc = rows[cur];
        const uint32_t* ic = ids[cur];
        if (!producer) {
            for (uint32_t i = ct; i < n; i += NC) {
                const uint32_t key = (rc[i * ST] >> (32 - SB - KB)) & (NKEY - 1);
                nxt[i] = (short)atomicExch(&head[key], (int)i);
            }
        } else if (threadIdx.x == 0) {
            nstaged[cur ^ 1] = 0;  // every read of it (item k - 1) happened before A
            staged_max = max(staged_max, got);
        }
        __syncthreads();  // B: chain links of the current item complete
        if (producer) {
            for (uint32_t i = threadIdx.x; i < NKEY; i += NP) head[i] = -1;  // chain building is over
            if (k + 1 < items) stage(k + 1, cur ^ 1);
        } else if constexpr (R == 9) {  // final round: equal d_8 and d_9 make a candidate
            for (uint32_t i = ct; i < n; i += NC) {
                // a level-8 payload is one word: slice, key and d_9 (CB = 8)
                const uint32_t di = rc[i * ST];
                int j = nxt[i], steps = 0;
                for (; j >= 0 && steps < EQ_MAX_CHAIN; j = nxt[j], ++steps) {
                    if (di != rc[(uint32_t)j * ST]) continue;
                    uint32_t* c = p.cands + (size_t)inst * (1 + 2 * EQ_MAX_CAND);
                    const uint32_t q = atomicAdd(&c[0], 1u);
                    if (q < EQ_MAX_CAND) {
                        c[1 + 2 * q] = ic[i];
                        c[2 + 2 * q] = ic[(uint32_t)j];
                    }
                }
                truncated += j >= 0;  // the chain went on past EQ_MAX_CHAIN: pairs not tried
            }
        } else {
            constexpr int WO = eqc_words(R), MO = eqc_payload(R);
            constexpr uint32_t REST = 0xFFFFFFFFu >> (SB + KB);  // payload bits after slice + key
            uint2* plog = (uint2*)p.pairs + ((size_t)inst * EQ_LEVELS + R) * (size_t)P * p.pmax;
            for (uint32_t i = ct; i < n; i += NC) {
                const uint32_t* ra = rc + i * ST;
                int j = nxt[i], steps = 0;
                for (; j >= 0 && steps < EQ_MAX_CHAIN; j = nxt[j], ++steps) {
                    const uint32_t* rb = rc + (uint32_t)j * ST;
                    uint32_t x[ST];
                    uint32_t rest = 0;
#pragma unroll
                    for (int q = 0; q < ST; ++q) {
                        x[q] = ra[q] ^ rb[q];
                        rest |= q ? x[q] : (x[q] & REST);
                    }
                    if (rest == 0) continue;  // identical remainder: only duplicate indices
                    const uint32_t nb = (x[0] >> 12) & (NCO - 1);  // the next digit's coarse bits
                    const uint32_t slot = atomicAdd(&cnt[nb], 1u);
                    const uint32_t kid = eqc_wave_alloc(&pcount);
                    if (kid >= p.pmax) {
                        ++lost_ids;
                        continue;
                    }
                    const uint32_t id = grp * p.pmax + kid;
                    plog[id] = make_uint2(ic[i], ic[(uint32_t)j]);
                    if (slot < p.seg) {
                        EqcRow<WO> r;
                        r.w[0] = id;
#pragma unroll
                        for (int q = 0; q < WO - 1; ++q)
                            r.w[1 + q] = q < MO ? (x[q] << 20) | (q + 1 < ST ? x[q + 1] >> 12 : 0u) : 0u;
                        *(EqcRow<WO>*)eqc_row<R>(p, inst, nb, grp, slot) = r;
                    }
                }
                truncated += j >= 0;
            }
        }
    }
    __syncthreads();
    // staging overflow (rows of a fine bucket beyond EQC_STAGE), segment overflow (level-R rows
    // beyond a segment) and pair ids beyond pmax are counted apart
    if (dropped) atomicAdd(&p.stats[inst * EQP_STATS + EQP_STAT_STAGE], dropped);
    if (threadIdx.x == 0 && staged_max) atomicMax(&p.stats[inst * EQP_STATS + EQP_STAT_STAGE_MAX], staged_max);
    if (lost_ids) atomicAdd(&p.stats[inst * EQP_STATS + EQC_STAT_PAIRS], lost_ids);
    if constexpr (R < 9) eqc_flush_counts(p, inst, grp, R, cnt);
    if (truncated) atomicAdd(&p.stats[inst * EQP_STATS + EQP_STAT_CHAIN], truncated);
}

// One 1024-thread workgroup per CU (4 waves per SIMD): at most 128 VGPRs.
#define EQC_ROUND_KERNEL(R) \
    extern "C" __global__ __launch_bounds__(EQC_BLOCK, EQC_MIN_WAVES) void eqc_round##R(EquihashCbDev p) { eqc_round_impl<R>(p); }
EQC_ROUND_KERNEL(1)
EQC_ROUND_KERNEL(2)
EQC_ROUND_KERNEL(3)
EQC_ROUND_KERNEL(4)
EQC_ROUND_KERNEL(5)
EQC_ROUND_KERNEL(6)
EQC_ROUND_KERNEL(7)
EQC_ROUND_KERNEL(8)

extern "C" __global__ __launch_bounds__(EQC_BLOCK, EQC_MIN_WAVES) void eqc_final(EquihashCbDev p) { eqc_round_impl<9>(p); }

// Leaf indices of every candidate: pairs[8] .. pairs[1] from its two level-8 ids (shared body:
// equihash_device.hpp, with the pair log as the children lookup).
extern "C" __global__ __launch_bounds__(256) void eqc_reconstruct(EquihashCbDev p) {
    const uint32_t inst = blockIdx.y;
    const uint2* plog = (const uint2*)p.pairs + (size_t)inst * EQ_LEVELS * (size_t)p.groups * p.pmax;
    const size_t level_stride = (size_t)p.groups * p.pmax;
    eq_reconstruct_tree<256>(
        [&](int level, uint32_t s, uint32_t& a, uint32_t& b) {
            const uint2 v = plog[(size_t)level * level_stride + s];
            a = v.x;
            b = v.y;
        },
        p.cands + (size_t)inst * (1 + 2 * EQ_MAX_CAND), p.sols + (size_t)inst * (1 + EQ_MAX_SOL * 512));
}
