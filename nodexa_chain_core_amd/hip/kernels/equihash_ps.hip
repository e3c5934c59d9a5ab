// Equihash(200,9) Wagner solver for gfx950 with private slot segments (new; the reference has
// no Equihash — SURVEY §0.4 / Appendix D). CPU golden model: csrc/pow/equihash.cpp.
//
// Why a second solver. The global-slot solver (equihash.hip) appends every output row with a
// returning global atomicAdd on its bucket's counter, and its 4096 one-bucket workgroups per
// round each pay that round trip before their stores. Measured on MI355X (profiles/README r2d):
// removing the atomics alone changed nothing (the rounds are bound by the scattered row stores,
// two 16-byte requests per row), so this engine (1) stores each level's rows at their payload
// size (below) and (2) pipelines each workgroup's bucket sequence so that the gathers of the next
// bucket run beside the collisions of the current one.
//
// Why not global per-bucket slots with an instance's writers on one XCD, so that one L2 merges
// all writers' rows of a bucket (the L2 does merge different workgroups' stores into a line:
// profiles/README r4t)? Each row then needs a returning global atomic, atomics execute at the
// memory side, and they top out near 29.5 G/s against 47.7 G/s for private appends of 24-byte
// rows (r4v); built into this engine it took 13.6 ms per 16-solve window against 8.6 (r4w).
//
// What bounds it (profiles/README r3_equihash): a random row store costs one memory transaction
// whatever its size (tools/scatter_ceiling.hip: 22-24 G rows/s for 16-64 byte rows, against
// 145 G/s when 4 lanes write one 128-byte run), and a level's rows go to 4096 buckets from every
// workgroup, so no store instruction can cover two rows of one line. With stores left out a round
// takes half its time; the other half is the producers' staging latency, which the workgroup
// shape sets: 1024 threads with 7 producer waves per workgroup and 32 writers per level cut the
// 8-solve batch from 5.52 ms (512 threads, 2 producer waves, 64 writers) to 4.37 ms.
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
// Row format (every level L): word 0 = back-pointer (level 0: the leaf index), then the row's
// bits [20L + 12, 200) big-endian and contiguous — the "payload". Bits [20L, 20L + 12) are the
// bucket and live in the row's address. So payload bits [0, 8) are the sub-digit a round chains
// on, bits [8, 28) the next digit, and a row takes 1 + ceil((188 - 20L) / 32)
// words, padded to 8, 8, 6, 5, 5, 4, 4, 4, 2 for levels 0..8 (eqp_words; 180 bytes per row over
// the nine levels against 224 for 32 / 16-byte slots). Two same-bucket rows collide into
// XOR(payload) << 20.
//
// Layouts (num_inst = ni):
//   hashes [2][ni][BUCKETS][EQP_SLOTS][eqp_words(level)] u32  (levels alternate between two buffers)
//   counts [ni][LEVELS][P][BUCKETS] u8
//   refs   [ni][LEVELS][BUCKETS][EQP_REF_STRIDE] u32
// Overflowing segments or staging areas drop rows (counted in p.stats per level), and a chain of
// equal sub-digits longer than EQ_MAX_CHAIN is cut (counted in p.stats[EQP_STAT_CHAIN]); at
// C = 32 for a mean of 8 rows per segment, 1024 staged for a mean of 512 per bucket and 64 for a
// mean chain of 2 they are rare (a chain cap of 24 and a candidate cap of 4096 were not: 0.03 % and
// 0.2 % of nonces, profiles r3zb). The host (ops/equihash.py) re-solves an instance with any such
// count on the golden solver, so the solution set is exact either way.
#include "equihash_device.hpp"

#ifndef EQP_BLOCK
#define EQP_BLOCK 1024  // threads per workgroup (the launcher's `block`)
#endif
#ifndef EQP_MIN_WAVES
#define EQP_MIN_WAVES 4  // waves per SIMD the round kernels are register-limited for (4: 128 VGPRs)
#endif
#ifndef EQP_NP
#define EQP_NP 448  // producer threads of a round workgroup (7 of its 16 waves)
#endif

// Instance and writer of this workgroup in a (writers x instances) grid: blockIdx.y = instance
// spreads every instance over all 8 XCDs (XCD-local instances measured neutral, profiles/README r4c).
#define EQP_INST_GRP(inst, grp) const uint32_t inst = blockIdx.y, grp = blockIdx.x

// EQP_NO_ROW_STORE (measurement only, results invalid): the row stores compiled out, the rest of
// each kernel (gathers, chains, slot counters, back-pointer copies) unchanged -- what the rows'
// own stores cost in time and in EA write requests (profiles/README r4r).
#ifdef EQP_NO_ROW_STORE
#define EQP_ROW_STORE(...) \
    do {                   \
        (void)r;           \
    } while (0)
#else
#define EQP_ROW_STORE(...) __VA_ARGS__
#endif

// Payload words of a level-`level` row: 6, 6, 5, 4, 4, 3, 3, 2, 1.
constexpr int eqp_payload(int level) { return (188 - 20 * level + 31) / 32; }
// Words per row slot in global memory: the payload plus the back-pointer, except that a 28-byte
// row is padded to 32 and a 12-byte one to 16 (measured r3j: 28-byte rows made round 1 slower
// and 12-byte rows rounds 7-8, while 24- and 20-byte rows made rounds 3-5 faster).
constexpr int eqp_words(int level) {
    return eqp_payload(level) == 6 ? 8 : eqp_payload(level) == 2 ? 4 : 1 + eqp_payload(level);
}
// LDS words per staged row: a 3-word payload is padded to 4 (one ds_read_b128 per row).
constexpr int eqp_lds_stride(int level) { return eqp_payload(level) == 3 ? 4 : eqp_payload(level); }

template <int N>
struct __attribute__((aligned(4))) EqpRow {
    uint32_t w[N];
};

// Word offset of a row slot of `level` (buffer level & 1); a segment's rows are contiguous.
template <int L>
NX_DEV size_t eqp_hidx(const EquihashPsDev& p, uint32_t inst, uint32_t bucket, uint32_t grp, uint32_t slot) {
    const size_t buf_words = (size_t)p.num_inst * EQ_BUCKETS * EQP_SLOTS * EQ_WORDS;  // one level buffer
    const size_t row = ((size_t)inst * EQ_BUCKETS + bucket) * EQP_SLOTS + grp * p.seg + slot;
    return (size_t)(L & 1) * buf_words + row * eqp_words(L);
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
NX_DEV void eqp_flush_counts(const EquihashPsDev& p, uint32_t inst, uint32_t grp, int level, const uint32_t* cnt2,
                             uint32_t dropped) {
    uint32_t* out = (uint32_t*)(p.counts + (((size_t)inst * EQ_LEVELS + level) * p.groups + grp) * EQ_BUCKETS);
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
    EQP_INST_GRP(inst, grp);
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
            const uint32_t nb = w[1] >> 20;  // bits [0, 12)
            const uint32_t slot = eqp_take_slot(cnt2, nb);
            if (slot < p.seg) {
                EqpRow<eqp_words(0)> r;
                r.w[0] = 2 * g + half;
#pragma unroll
                for (int k = 0; k < eqp_words(0) - 1; ++k)
                    r.w[1 + k] = k < eqp_payload(0) ? (w[k + 1] << 12) | (w[k + 2] >> 20) : 0u;
                EQP_ROW_STORE(*(EqpRow<eqp_words(0)>*)(p.hashes + eqp_hidx<0>(p, inst, nb, grp, slot)) = r);
            }
        }
    }
    __syncthreads();
    eqp_flush_counts(p, inst, grp, 0, cnt2, 0);
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
// level L into LDS rows (payload words at stride ST = eqp_lds_stride(L), zero padded) and copy their
// back-pointers to refs[L][b][pos]. A row's segment is found by binary search over the prefix
// segc, so every load is a real row (about 4 per producer lane per bucket, all in flight together).
template <int L, uint32_t NP>
NX_DEV void eqp_gather_rows(const EquihashPsDev& p, uint32_t inst, uint32_t b, const uint32_t* segc,
                            uint32_t n, uint32_t* rows, uint32_t pt) {
    constexpr int BATCH = 4, W = eqp_words(L), PL = eqp_payload(L), ST = eqp_lds_stride(L);
    const uint32_t P = p.groups;
    uint32_t* refs = p.refs + (((size_t)inst * EQ_LEVELS + L) * EQ_BUCKETS + b) * EQP_REF_STRIDE;
#pragma unroll 1
    for (uint32_t p0 = pt; p0 < n; p0 += NP * BATCH) {
        EqpRow<W> r[BATCH];
#pragma unroll
        for (int k = 0; k < BATCH; ++k) {
            const uint32_t pos = p0 + k * NP;
            if (pos >= n) continue;
            uint32_t a = 0, z = P;  // largest segment whose prefix is <= pos
            while (z - a > 1) {
                const uint32_t mid = (a + z) >> 1;
                if (segc[mid] <= pos) a = mid; else z = mid;
            }
            r[k] = *(const EqpRow<W>*)(p.hashes + eqp_hidx<L>(p, inst, b, a, pos - segc[a]));
        }
#pragma unroll
        for (int k = 0; k < BATCH; ++k) {
            const uint32_t pos = p0 + k * NP;
            if (pos >= n) continue;
            refs[pos] = r[k].w[0];
#pragma unroll
            for (int q = 0; q < ST; ++q) rows[pos * ST + q] = q < PL ? r[k].w[1 + q] : 0u;
        }
    }
}

// Round R (1..8): collide level R-1 on digit R-1 bucket by bucket, write level R. R = 9 is the
// final round: level-8 rows colliding on d_8 and d_9 (40 bits) become candidates.
//
// Producer / consumer split: the first EQP_NP threads (7 waves) stage the NEXT bucket (count
// scan, row gathers into the other LDS row buffer, back-pointer copies, the counts of the bucket
// after that) while the other 9 waves chain and collide the current bucket and emit rows. A wave's
// vmcnt counts its loads and stores together in issue order, so keeping the gathers out of the
// emitting waves means no load ever waits behind a scattered row store; the gathers' latency
// hides behind the collisions.
// Two barriers per bucket: after staging (A: rows ready) and after chaining (B: links ready).
template <int R>
NX_DEV void eqp_round_impl(const EquihashPsDev& p) {
    constexpr int ST = eqp_lds_stride(R - 1);  // LDS words per staged level-(R-1) row
    constexpr uint32_t NP = EQP_NP, NC = EQP_BLOCK - NP;  // producer / consumer threads
    __shared__ uint32_t cnt2[EQ_BUCKETS / 2];
    __shared__ __attribute__((aligned(16))) uint32_t rows[2][EQP_STAGE * ST];
    __shared__ int head[256];
    __shared__ short nxt[EQP_STAGE];
    __shared__ uint32_t segc[NP / 64][256];  // one prefix copy per producer wave (no cross-wave sync)
    __shared__ uint32_t nstaged[2];
    // P = writers per level (the counts layout); the workgroups stride over the buckets by the
    // grid width, which is P for rounds 1..8 (workgroup = writer) and wider for the final round
    EQP_INST_GRP(inst, grp);
    const uint32_t P = p.groups, G = gridDim.x;
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
        eqp_gather_rows<R - 1, NP>(p, inst, bk, my_segc, n, rows[buf], threadIdx.x);
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
                const uint32_t sub = rc[i * ST] >> 24;
                nxt[i] = (short)atomicExch(&head[sub], (int)i);
            }
        }
        __syncthreads();  // B: chain links of the current bucket complete
        if (producer) {
            for (uint32_t i = threadIdx.x; i < 256; i += NP) head[i] = -1;  // chain building is over
            if (b + G < EQ_BUCKETS) stage(b + G, cur ^ 1);
        } else if constexpr (R == 9) {  // final round: equal d_8 (chain) and d_9 make a candidate
            for (uint32_t i = ct; i < n; i += NC) {
                // a level-8 payload is one word: the low bits of d_8, d_9, zero padding
                const uint32_t di = rc[i * ST];
                int j = nxt[i], steps = 0;
                for (; j >= 0 && steps < EQ_MAX_CHAIN; j = nxt[j], ++steps) {
                    if (di != rc[(uint32_t)j * ST]) continue;
                    uint32_t* c = p.cands + (size_t)inst * (1 + 2 * EQ_MAX_CAND);
                    const uint32_t k = atomicAdd(&c[0], 1u);
                    if (k < EQ_MAX_CAND) {
                        c[1 + 2 * k] = b * EQP_REF_STRIDE + i;
                        c[2 + 2 * k] = b * EQP_REF_STRIDE + (uint32_t)j;
                    }
                }
                truncated += j >= 0;  // the chain went on past EQ_MAX_CHAIN: pairs not tried
            }
        } else {
            constexpr int WO = eqp_words(R), MO = eqp_payload(R);
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
                        rest |= q ? x[q] : (x[q] & 0x00FFFFFFu);
                    }
                    if (rest == 0) continue;  // identical remainder: only duplicate indices
                    const uint32_t nb = (x[0] >> 12) & 0xFFFu;
                    const uint32_t slot = eqp_take_slot(cnt2, nb);
                    if (slot < p.seg) {
                        EqpRow<WO> r;
                        r.w[0] = (b << 20) | (i << 10) | (uint32_t)j;
#pragma unroll
                        for (int q = 0; q < WO - 1; ++q)
                            r.w[1 + q] = q < MO ? (x[q] << 20) | (q + 1 < ST ? x[q + 1] >> 12 : 0u) : 0u;
                        EQP_ROW_STORE(*(EqpRow<WO>*)(p.hashes + eqp_hidx<R>(p, inst, nb, grp, slot)) = r);
                    }
                }
                truncated += j >= 0;  // the chain went on past EQ_MAX_CHAIN: pairs not tried
            }
        }
    }
    __syncthreads();
    // staging overflow (rows of a level-(R-1) bucket beyond EQP_STAGE) and segment overflow (level R
    // rows beyond a segment) are counted apart
    if (dropped) atomicAdd(&p.stats[inst * EQP_STATS + EQP_STAT_STAGE], dropped);
    if (threadIdx.x == 0) atomicMax(&p.stats[inst * EQP_STATS + EQP_STAT_STAGE_MAX], staged_max);
    if constexpr (R < 9) eqp_flush_counts(p, inst, grp, R, cnt2, 0);
    if (truncated) atomicAdd(&p.stats[inst * EQP_STATS + EQP_STAT_CHAIN], truncated);
}

// One 1024-thread workgroup per CU (4 waves per SIMD): at most 128 VGPRs.
#define EQP_ROUND_KERNEL(R) \
    extern "C" __global__ __launch_bounds__(EQP_BLOCK, EQP_MIN_WAVES) void eqp_round##R(EquihashPsDev p) { eqp_round_impl<R>(p); }
EQP_ROUND_KERNEL(1)
EQP_ROUND_KERNEL(2)
EQP_ROUND_KERNEL(3)
EQP_ROUND_KERNEL(4)
EQP_ROUND_KERNEL(5)
EQP_ROUND_KERNEL(6)
EQP_ROUND_KERNEL(7)
EQP_ROUND_KERNEL(8)

extern "C" __global__ __launch_bounds__(EQP_BLOCK, EQP_MIN_WAVES) void eqp_final(EquihashPsDev p) { eqp_round_impl<9>(p); }

// Leaf indices of every candidate (shared body: equihash_device.hpp).
extern "C" __global__ __launch_bounds__(256) void eqp_reconstruct(EquihashPsDev p) {
    const uint32_t inst = blockIdx.y;
    eq_reconstruct_body<EQP_REF_STRIDE, 256>(p.refs + (size_t)inst * EQ_LEVELS * EQ_BUCKETS * EQP_REF_STRIDE,
                                             p.cands + (size_t)inst * (1 + 2 * EQ_MAX_CAND),
                                             p.sols + (size_t)inst * (1 + EQ_MAX_SOL * 512));
}
