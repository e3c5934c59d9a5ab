// Equihash(200,9) Wagner solver for gfx950 with coarse destination buckets (new; the reference has
// no Equihash — SURVEY §0.4 / Appendix D). CPU golden model: csrc/pow/equihash.cpp.
//
// What bounds a Wagner round on MI355X is its scattered row stores: every round appends 2^21 rows
// per instance to random buckets, and with 4096 destination buckets each row leaves the L2 as its
// own partial-line write (1.06-1.18 EA write requests per row, profiles/README r4r/r4l); the
// private-slot solver (equihash_ps.hip) sits on that floor. This solver keeps its collision
// structure -- 4096 fine buckets of ~512 rows staged in LDS, 8-bit chain sub-digits, 32-bit
// back-pointers (bucket << 20 | index a << 10 | index b) and the refs table -- but STORES a level's
// rows by the top EQC_COARSE_BITS (8) bits of their next digit only: a writer appends to 256
// segments instead of 4096, and the L2 merges its appends into lines before they go out
// (tools/eq_runs_probe.hip, profiles r5a: 0.43-0.54 requests and 0.32-0.44 ms per 33.5M rows at 256
// buckets against 1.06-1.18 and 0.71-0.87 ms at 4096). The remaining 4 bucket bits (the slice)
// travel in the row.
//
// So a coarse bucket holds 16 fine buckets. The workgroup that owns it stages them one after
// another in two phases (profiles r5c: one pass over the coarse bucket per fine bucket costs more
// than the stores save): phase 1, once per coarse bucket, reads only word 1 of every row (the slice
// bits) with all of a lane's positions in flight at once and keeps (segment, slice) per position in
// registers; phase 2, per fine bucket, gives each wave one contiguous range of staging indices for
// the rows of its positions in that slice (one LDS atomic), parks their (segment, slot) there, and
// loads those rows spread evenly over the wave's lanes.
//
// Row format (level L): word 0 = back-pointer (level 0: the leaf index), then the row's bits
// [20L + 8, 200) big-endian and contiguous (payload: slice [0, 4), chain sub-digit [4, 12), the
// next digit's coarse bits [12, 20), ...). Bits [20L, 20L + 8) are the coarse bucket and live in
// the row's address. Payload words 6, 6, 5, 5, 4, 3, 3, 2, 1 for levels 0..8.
//
// Layouts (num_inst = ni, P writers per instance, seg rows per segment: mean 2^13 / P + 8 sigma):
//   hashes [2][ni][COARSE][P][seg][words(level)]   (levels alternate between two buffers)
//   counts [ni][LEVELS][P][COARSE] u16
//   refs   [ni][LEVELS][4096][EQP_REF_STRIDE]       (as equihash_ps.hip: staged order, fine buckets)
// Every device-side cap (segment slots, positions per lane, staged rows, chain length, candidates)
// is counted in p.stats; the host re-solves an instance with any count on the golden solver, so
// the solution set is exact either way (ops/equihash.py).
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
#ifndef EQC_KMAX
#define EQC_KMAX 24  // coarse-bucket positions per producer lane: 24 x 448 = 10752 rows (mean 8.2-8.6k)
#endif
#ifndef EQC_B2
#define EQC_B2 4  // kept rows in flight per lane in phase 2 (a slice is ~512 rows: ~0.7 per lane)
#endif

constexpr uint32_t CB = EQC_COARSE_BITS, SB = EQ_BUCKET_BITS - CB, KB = 8;
constexpr uint32_t NCO = EQC_COARSE, NSL = 1u << SB;
static_assert(CB >= 8 && CB <= 11, "a level-8 payload must fit one word and a slice take 1..4 bits");

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
// workgroup's segment of their coarse bucket (word 0 = the leaf index).
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

// Phase 1, once per coarse bucket d: for this lane's positions pt + k * NP (k < KMAX) of the
// bucket's rows (its P segments as one list of `total` rows), meta = segment << 8 | slice (16 bits
// per position, two per word), read from word 1 of each row; positions past `total` get slice
// 0xFF. The segment of increasing positions is found by walking the prefix segc forward.
template <int L, uint32_t NP>
NX_DEV void eqc_scan_slices(const EquihashCbDev& p, uint32_t inst, uint32_t d, const uint32_t* segc, uint32_t total,
                            uint32_t (&meta)[(EQC_KMAX + 1) / 2]) {
    constexpr int K = EQC_KMAX;
    const uint32_t pt = threadIdx.x, P = p.groups;
    uint32_t w1[K], seg[K];
    uint32_t a = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t pos = pt + (uint32_t)k * NP;
        w1[k] = 0xFFFFFFFFu;
        seg[k] = a;
        if (pos < total) {
            while (a + 1 < P && segc[a + 1] <= pos) ++a;
            seg[k] = a;
            w1[k] = eqc_row<L>(p, inst, d, a, pos - segc[a])[1];
        }
    }
#pragma unroll
    for (int k = 0; k < (K + 1) / 2; ++k) meta[k] = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t pos = pt + (uint32_t)k * NP;
        const uint32_t sl = pos < total ? w1[k] >> (32 - SB) : 0xFFu;
        meta[k / 2] |= ((seg[k] << 8) | sl) << (16 * (k & 1));
    }
}

// Phase 2: stage fine bucket b = d * NSL + s (slice s of coarse bucket d): the rows of this lane's
// positions in the slice get staging indices from one contiguous range per wave, the wave parks
// their (segment, slot) there and loads the range's rows spread evenly over its 64 lanes; payload
// words to `rows` (stride ST), back-pointers to refs[L][b][index]. Returns the rows dropped at the
// staging cap.
template <int L, uint32_t NP>
NX_DEV uint32_t eqc_stage_slice(const EquihashCbDev& p, uint32_t inst, uint32_t d, uint32_t s, const uint32_t* segc,
                                const uint32_t (&meta)[(EQC_KMAX + 1) / 2], uint32_t* rows, uint32_t* park,
                                uint32_t* nstaged) {
    constexpr int K = EQC_KMAX, B2 = EQC_B2, W = eqc_words(L), PL = eqc_payload(L), ST = eqc_lds_stride(L);
    const uint32_t pt = threadIdx.x, lane = eqc_lane();
    uint32_t nk = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) nk += ((meta[k / 2] >> (16 * (k & 1))) & 0xFFu) == s;
    uint32_t x = nk;  // wave prefix of the kept counts: one range per wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if ((int)lane >= o) x += y;
    }
    const uint32_t wave_tot = __shfl(x, 63, 64);
    uint32_t base = 0;
    if (lane == 0 && wave_tot) base = atomicAdd(nstaged, wave_tot);
    base = __shfl(base, 0, 64);
    uint32_t at = base + x - nk;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t m = (meta[k / 2] >> (16 * (k & 1))) & 0xFFFFu;
        if ((m & 0xFFu) == s) {
            const uint32_t a = m >> 8, pos = pt + (uint32_t)k * NP;
            if (at < EQP_STAGE) park[at] = (a << 16) | (pos - segc[a]);
            ++at;
        }
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t n = base >= EQP_STAGE ? 0 : min(wave_tot, (uint32_t)EQP_STAGE - base);
    const uint32_t b = d * NSL + s;
    uint32_t* refs = p.refs + (((size_t)inst * EQ_LEVELS + L) * EQ_BUCKETS + b) * EQP_REF_STRIDE;
#pragma unroll 1
    for (uint32_t t0 = 0; t0 < n; t0 += 64 * B2) {
        EqcRow<W> r[B2];
        uint32_t idx[B2];
#pragma unroll
        for (int q = 0; q < B2; ++q) {
            const uint32_t t = t0 + lane + 64u * q;
            idx[q] = t < n ? base + t : 0xFFFFFFFFu;
            if (idx[q] == 0xFFFFFFFFu) continue;
            const uint32_t pk = park[idx[q]];
            r[q] = *(const EqcRow<W>*)eqc_row<L>(p, inst, d, pk >> 16, pk & 0xFFFFu);
        }
#pragma unroll
        for (int q = 0; q < B2; ++q) {
            if (idx[q] == 0xFFFFFFFFu) continue;
            refs[idx[q]] = r[q].w[0];
#pragma unroll
            for (int w = 0; w < ST; ++w) rows[idx[q] * ST + w] = w < PL ? r[q].w[1 + w] : 0u;
        }
    }
    return lane == 0 ? wave_tot - n : 0u;
}

// Round R (1..8): collide level R-1 on digit R-1 fine bucket by fine bucket, write level R.
// R = 9 is the final round: level-8 rows equal on d_8 and d_9 (40 bits) become candidates.
//
// Producer / consumer split as in the private-slot solver: the first EQC_NP threads (7 waves)
// stage the NEXT fine bucket while the other 9 waves chain and collide the current one and emit
// rows. Two barriers per fine bucket: after staging (A: rows ready) and after chaining (B: links
// ready).
template <int R>
NX_DEV void eqc_round_impl(const EquihashCbDev& p) {
    constexpr int ST = eqc_lds_stride(R - 1);  // LDS words per staged level-(R-1) row
    constexpr uint32_t NP = EQC_NP, NC = EQC_BLOCK - NP;
    __shared__ uint32_t cnt[NCO];
    __shared__ __attribute__((aligned(16))) uint32_t rows[2][EQP_STAGE * ST];
    __shared__ uint32_t park[EQP_STAGE];
    __shared__ int head[1 << KB];
    __shared__ short nxt[EQP_STAGE];
    __shared__ uint32_t segc[NP / 64][EQC_MAX_P];  // one prefix copy per producer wave
    __shared__ uint32_t nstaged[2];
    if (p.coarse != NCO) return;  // geometry mismatch (whole workgroup): nothing staged or emitted
    const uint32_t inst = blockIdx.y, grp = blockIdx.x;
    const uint32_t P = p.groups, G = gridDim.x;
    const bool producer = threadIdx.x < NP;
    const uint32_t ct = threadIdx.x - NP;
    uint32_t* my_segc = segc[threadIdx.x / 64 % (NP / 64)];
    eqc_clear(cnt);
    for (uint32_t i = threadIdx.x; i < (1u << KB); i += EQC_BLOCK) head[i] = -1;
    if (threadIdx.x == 0) nstaged[0] = nstaged[1] = 0;
    __syncthreads();
    // work item k of this workgroup: coarse bucket grp + G * (k / NSL), slice k % NSL (a coarse
    // bucket's fine buckets back to back, so its phase-1 scan serves all of them)
    const uint32_t items = grp < NCO ? ((NCO - 1 - grp) / G + 1) * NSL : 0;
    auto coarse = [&](uint32_t k) { return grp + G * (k / NSL); };
    uint32_t cv[4] = {0, 0, 0, 0};
    uint32_t meta[(EQC_KMAX + 1) / 2];
    uint32_t dropped = 0, truncated = 0, staged_max = 0;
    auto stage = [&](uint32_t k, uint32_t buf) {
        const uint32_t d = coarse(k), s = k % NSL;
        if (s == 0) {
            const uint32_t total = eqc_wave_scan(P, cv, my_segc);  // counts loaded one bucket ahead
            if (total > NP * EQC_KMAX && threadIdx.x == 0) dropped += total - NP * EQC_KMAX;
            eqc_scan_slices<R - 1, NP>(p, inst, d, my_segc, total, meta);
            if (k + NSL < items) eqc_load_counts(p, inst, R - 1, coarse(k + NSL), cv);
        }
        dropped += eqc_stage_slice<R - 1, NP>(p, inst, d, s, my_segc, meta, rows[buf], park, &nstaged[buf]);
    };
    if (producer && items) {  // prologue: stage the first item
        eqc_load_counts(p, inst, R - 1, coarse(0), cv);
        stage(0, 0);
    }
    uint32_t cur = 0;
    for (uint32_t k = 0; k < items; ++k, cur ^= 1) {
        __syncthreads();  // A: rows[cur] staged, head reset, previous item's emission done
        const uint32_t got = nstaged[cur];
        const uint32_t n = min(got, (uint32_t)EQP_STAGE);
        const uint32_t* rc = rows[cur];
        const uint32_t b = coarse(k) * NSL + k % NSL;  // the fine bucket being collided
        if (!producer) {
            for (uint32_t i = ct; i < n; i += NC) {
                const uint32_t sub = (rc[i * ST] >> (32 - SB - KB)) & ((1u << KB) - 1);
                nxt[i] = (short)atomicExch(&head[sub], (int)i);
            }
        } else if (threadIdx.x == 0) {
            nstaged[cur ^ 1] = 0;  // every read of it (item k - 1) happened before A
            staged_max = max(staged_max, got);
        }
        __syncthreads();  // B: chain links of the current item complete
        if (producer) {
            for (uint32_t i = threadIdx.x; i < (1u << KB); i += NP) head[i] = -1;  // chain building is over
            if (k + 1 < items) stage(k + 1, cur ^ 1);
        } else if constexpr (R == 9) {  // final round: equal d_8 (chain) and d_9 make a candidate
            for (uint32_t i = ct; i < n; i += NC) {
                // a level-8 payload is one word: slice, sub-digit and d_9 (CB = 8)
                const uint32_t di = rc[i * ST];
                int j = nxt[i], steps = 0;
                for (; j >= 0 && steps < EQ_MAX_CHAIN; j = nxt[j], ++steps) {
                    if (di != rc[(uint32_t)j * ST]) continue;
                    uint32_t* c = p.cands + (size_t)inst * (1 + 2 * EQ_MAX_CAND);
                    const uint32_t q = atomicAdd(&c[0], 1u);
                    if (q < EQ_MAX_CAND) {
                        c[1 + 2 * q] = b * EQP_REF_STRIDE + i;
                        c[2 + 2 * q] = b * EQP_REF_STRIDE + (uint32_t)j;
                    }
                }
                truncated += j >= 0;  // the chain went on past EQ_MAX_CHAIN: pairs not tried
            }
        } else {
            constexpr int WO = eqc_words(R), MO = eqc_payload(R);
            constexpr uint32_t REST = 0xFFFFFFFFu >> (SB + KB);  // payload bits after slice + sub-digit
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
                    if (slot < p.seg) {
                        EqcRow<WO> r;
                        r.w[0] = (b << 20) | (i << 10) | (uint32_t)j;
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
    // staging overflow (rows of a fine bucket beyond EQP_STAGE, or of a coarse bucket beyond the
    // positions the producers scan) and segment overflow (level-R rows beyond a segment) apart
    if (dropped) atomicAdd(&p.stats[inst * EQP_STATS + EQP_STAT_STAGE], dropped);
    if (threadIdx.x == 0 && staged_max) atomicMax(&p.stats[inst * EQP_STATS + EQP_STAT_STAGE_MAX], staged_max);
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

// Leaf indices of every candidate (shared body: equihash_device.hpp; refs as equihash_ps.hip).
extern "C" __global__ __launch_bounds__(256) void eqc_reconstruct(EquihashCbDev p) {
    const uint32_t inst = blockIdx.y;
    eq_reconstruct_body<EQP_REF_STRIDE, 256>(p.refs + (size_t)inst * EQ_LEVELS * EQ_BUCKETS * EQP_REF_STRIDE,
                                             p.cands + (size_t)inst * (1 + 2 * EQ_MAX_CAND),
                                             p.sols + (size_t)inst * (1 + EQ_MAX_SOL * 512));
}
