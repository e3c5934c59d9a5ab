// Kernel parameter blocks shared by the gfx950 kernels (device side) and the
// HIP host runtime (hip/runtime/*.cpp). Every kernel takes exactly one of these
// structs by value; the host passes it through hipModuleLaunchKernel's
// HIP_LAUNCH_PARAM_BUFFER_POINTER, so the layout here is the ABI.
#pragma once
#include <stdint.h>

#define NODEXA_KAWPOW_MAX_SHARES 64
#define NODEXA_KAWPOW_BLOCK 256

// Fast u32 modulo by a runtime constant d (round-up multiply-shift, valid for
// every 32-bit numerator): q = (mulhi(x, m) + ((x - mulhi(x, m)) >> 1)) >> (s - 1).
struct FastMod32 {
    uint32_t d;
    uint32_t m;
    uint32_t s;  // ceil(log2 d), >= 1
    uint32_t mb; // floor(2^32 / d): Barrett estimate, off by at most one d (one min() fixes it)
    uint32_t m24; // floor(2^40 / d) for 2^16 < d < 2^24 (else 0; 2^40/2^16 needs 25 bits): 24-bit Barrett, see kawpow_search.hip
    uint32_t pad;
};

struct EthashDagParams {
    const void* light;     // light cache, light_items x 64 B
    void* dag;             // output, 512-bit items
    uint64_t first_item;   // first 512-bit item to compute
    uint64_t num_items;    // number of 512-bit items in this launch
    uint32_t light_items;  // light cache items (prime)
    uint32_t pad;
};

struct KawpowShare {
    uint64_t nonce;
    uint32_t mix[8];    // mix digest words (storage order)
    uint32_t final_[8]; // final hash words (storage order)
};

struct KawpowResults {
    uint32_t count;     // number of shares appended (may exceed MAX; extra dropped)
    uint32_t skipped;   // workgroups that found their launch stale (generation moved on) and searched nothing
    uint32_t pad[2];
    struct KawpowShare shares[NODEXA_KAWPOW_MAX_SHARES];
};

struct KawpowSearchParams {
    const void* dag;           // 2048-bit items (16 x uint4 each)
    struct KawpowResults* results;
    uint64_t start_nonce;
    uint64_t target;           // share if bswap64(final[0..1]) <= target (upper 64 bits, BE)
    uint32_t header[8];        // header hash words (storage order)
    struct FastMod32 items;    // modulo by number of 2048-bit items (full_items / 2)
    uint32_t* scratch;         // >= 8 words per nonce of the launch (variants that park digests in HBM)
    // Stale-work abort: each workgroup reads *gen_word (host-mapped, written by the miner when the
    // template changes) once at its start and searches nothing if it differs from `generation`.
    const uint32_t* gen_word;  // nullptr: never abort
    uint32_t generation;
    uint32_t pad;
};

// Light-mode / full-DAG batch verification of (header, nonce) pairs.
struct KawpowVerifyJob {
    uint32_t header[8];
    uint64_t nonce;
    uint32_t block_number;
    uint32_t pad;
};

// ---------------------------------------------------------------- Equihash(200,9)
#define EQ_BUCKET_BITS 12
#define EQ_BUCKETS (1 << EQ_BUCKET_BITS)
#define EQ_WORDS 8
#define EQ_LEVELS 9
#define EQ_MAX_CAND 16384  // ~500-1100 final-round collisions per nonce (almost all duplicate trees), 4300-4900
                          // in ~0.2 % of nonces: a 4096 cap sent those to the host re-solve (profiles r3zb)
#define EQ_RECON_GROUPS 128  // reconstruct workgroups per instance (grid-stride over candidates)
#define EQ_MAX_SOL 16


// Private-slot Equihash(200,9) solver (equihash_ps.hip). Each round runs `groups` (P)
// workgroups per instance; workgroup w owns a `seg`-row (C) segment of every bucket of the
// level it writes and allocates its slots with LDS atomics, so no global atomic is issued per
// row (the global-slot solver's per-row atomics execute at the memory side and bound its
// rounds: profiles/README r2c). P * C = EQP_SLOTS rows of address space per bucket.
#define EQP_SLOTS 2048
#define EQP_STAGE 1024     // rows of one bucket staged in LDS (mean 512-560; the 10-bit staged index caps it)
#define EQP_REF_STRIDE 1024  // refs per bucket: a 10-bit staged index
#define EQP_STATS 16
#define EQP_STAT_CHAIN 9   // stats slot: chains cut at EQ_MAX_CHAIN (slots 0-8: segment overflow per level)
#define EQP_STAT_STAGE 10  // rows beyond EQP_STAGE in a staged bucket (any round)
#define EQP_STAT_STAGE_MAX 11  // largest bucket seen by a round (diagnostic, not a loss)
#define EQP_FINAL_GROUPS 1024  // final-round workgroups per instance (it writes no level)
struct EquihashPsDev {
    const uint64_t* msgs;   // [inst][16] BLAKE2b message words (input bytes, LE; the index is OR-ed in-kernel)
    uint64_t h0[8];
    uint32_t input_len;
    uint32_t num_inst;
    uint32_t groups;        // P: workgroups per instance per round (a power of two <= 256)
    uint32_t seg;           // C: rows per (bucket, workgroup) segment, EQP_SLOTS / P
    uint32_t* hashes;       // [2][inst][BUCKETS][P][C][WORDS]: word 0 = back-pointer, 1..7 = row
    uint32_t* refs;         // [inst][LEVELS][BUCKETS][EQP_REF_STRIDE] in staged (compact) order
    uint8_t* counts;        // [inst][LEVELS][P][BUCKETS] rows per segment (clamped to C)
    uint32_t* cands;        // [inst][1 + 2*MAX_CAND]: count, then (bucket << 10 | index) pairs at level 8
    uint32_t* sols;         // [inst][1 + MAX_SOL*512]
    uint32_t* stats;        // [inst][EQP_STATS]: rows dropped per level (segment or staging overflow)
};

// Batch ECDSA verification (secp256k1_verify.hip): one job per signature, limbs little-endian.
#define SECP_KIND_UNCOMPRESSED 0u  // y given, checked on the curve
#define SECP_KIND_EVEN 2u          // compressed, y recovered with even parity
#define SECP_KIND_ODD 3u           // compressed, odd parity
#define SECP_KIND_INVALID 0xffu    // host parsing already failed: result 0
struct SecpVerifyJob {
    uint32_t x[8], y[8];  // public key
    uint32_t r[8], s[8];  // signature, s normalised to low-S, both in [0, n)
    uint32_t z[8];        // message hash as a 256-bit big-endian integer (reduced mod n in-kernel)
    uint32_t kind;
    uint32_t pad[3];
};
struct SecpVerifyParams {
    const struct SecpVerifyJob* jobs;
    const uint32_t* gtab;  // 64 x 16 affine points j * 16^i * G, 16 limbs (x then y) each
    uint32_t* out;         // per job: 1 valid, 0 invalid, 2 degenerate case (re-check on the host)
    uint32_t n;
    uint32_t pad;
};

// Batch verification of packed Equihash(200,9) solutions (equihash.hip eq_verify).
#define EQ_SOL_WORDS 336  // 1344 bytes = 512 x 21-bit big-endian indices
struct EquihashVerifyParams {
    const uint64_t* msgs;   // [num][16] BLAKE2b message words of each input (as EquihashPsDev)
    uint64_t h0[8];
    uint32_t input_len;
    uint32_t num;
    const uint32_t* sols;   // [num][EQ_SOL_WORDS] packed solutions
    uint32_t* out;          // [num] 0 = valid, else the failing rule (EQ_V_*)
};
// The solver's own solution slots, verified on the device (equihash.hip eq_verify_slots).
struct EquihashSlotVerifyParams {
    const uint64_t* msgs;   // [inst][16] BLAKE2b message words (as EquihashPsDev)
    uint64_t h0[8];
    uint32_t input_len;
    uint32_t num_inst;
    const uint32_t* sols;   // [inst][1 + EQ_MAX_SOL*512]: count, then unpacked indices
    uint32_t* out;          // [inst][EQ_MAX_SOL]: EQ_V_* per slot, EQ_V_EMPTY past the count
};
#define EQ_V_EMPTY 255
#define EQ_V_OK 0
#define EQ_V_COLLISION 1
#define EQ_V_ORDER 2
#define EQ_V_DUPLICATE 3
#define EQ_V_NONZERO 4

// Batch verification with the period program as data (kawpow_verify.hip).
#define KV_PROG_WORDS 64
struct KawpowVerifyParams {
    const void* dag;                    // full DAG of the batch's epoch (2048-bit items)
    const struct KawpowVerifyJob* jobs; // sorted by period, padded so each 64-job slab is one period
    const uint32_t* programs;           // [num_programs][KV_PROG_WORDS]
    const uint32_t* job_program;        // per 64-job slab: program index
    uint32_t* out;                      // per job: mix[8], final[8]
    uint32_t num_jobs;
    uint32_t pad;
    struct FastMod32 items;
};

// Light-mode batch verification (kawpow_verify_light.hip): no DAG, every DAG
// item a round touches is recomputed from the light cache. One job per 16-lane
// group; jobs may mix periods freely (each group loads its own program).
struct KawpowLightParams {
    const void* light;                  // light cache of the batch's epoch (512-bit items)
    const uint32_t* l1;                 // 4096-word L1 (first 16 KiB of the DAG, host-computed)
    const struct KawpowVerifyJob* jobs;
    const uint32_t* programs;           // [num_programs][KV_PROG_WORDS]
    const uint32_t* job_program;        // per job: program index
    uint32_t* out;                      // per job: mix[8], final[8]
    uint32_t num_jobs;
    uint32_t num_programs;
    struct FastMod32 light_items;       // modulo by the number of 512-bit light items
    struct FastMod32 items;             // modulo by the number of 2048-bit DAG items
    const void* dag;                    // kawpow_verify_dag: resident DAG (2048-bit items); else null
    const int32_t* slots;               // kawpow_verify_waves: job per 16-lane group slot, 4 slots per
                                        // wave, all of one period; -1 = idle group
    uint32_t num_slots;
    uint32_t pad;
};

struct KawpowHashParams {
    const void* dag;                  // full DAG (2048-bit items)
    const struct KawpowVerifyJob* jobs;
    uint32_t* out;                    // per job: mix[8] then final[8]
    uint32_t num_jobs;
    uint32_t pad;
    struct FastMod32 items;
};

// Classic Ethash hashimoto over the resident DAG (ethash_hashimoto.hip): jobs are (header hash,
// nonce) pairs (KawpowVerifyJob, block_number unused); out per job: mix[8] then final[8].
struct EthashHashParams {
    const void* dag;                  // full dataset (1024-bit pages = pairs of 512-bit items)
    const struct KawpowVerifyJob* jobs;
    uint32_t* out;
    uint32_t* seeds;                  // scratch: n x 16 words (keccak512 seeds, phase 1 -> 2, 3)
    uint32_t num_jobs;
    uint32_t max_hits;                // search: capacity of hits[1..]
    struct FastMod32 pages;           // modulo by the number of 1024-bit pages (full_items)
    // search mode (jobs == nullptr): job i hashes (header, start_nonce + i); with `hits`, the final
    // kernel appends i for every final <= boundary (both big-endian byte strings, 8 words each)
    uint32_t header[8];
    uint64_t start_nonce;
    uint32_t boundary[8];
    uint32_t* hits;                   // [0] = count, [1..max_hits] = job indices
};

// X16R / X16RV2 chain step on the GPU (x16r.hip): workgroup (x, slot) runs slot `blockIdx.y` over
// its share of the headers whose step-`step` algorithm is that slot.
struct X16rStepParams {
    const uint8_t* headers;     // n x 80 bytes (the legacy header)
    uint8_t* state;             // n x 64 bytes: the chain value, the final hash in its first 32
    const uint8_t* v2;          // n flags: X16RV2 (Tiger pre-hash on slots 4, 6, 15)
    const int32_t* order;       // this step's header indices grouped by slot
    const int32_t* offsets;     // 17 entries: slot a owns order[offsets[a] .. offsets[a + 1])
    uint32_t n;
    uint32_t step;              // 0: hash the 80-byte header, else the 64-byte chain value
    // search mode (tmpl != nullptr): header i is the 80-byte template with nNonce (bytes 76..79,
    // little-endian) = start_nonce + i, and v2_all replaces the per-header flags
    const uint8_t* tmpl;
    uint32_t start_nonce;
    uint32_t v2_all;
};

// x16r_hits: the lowest index i < n whose chain value (a little-endian uint256 in its first 32
// bytes) is <= target, by atomicMin into *best (the host sets it to 0xffffffff first).
struct X16rHitParams {
    const uint8_t* state;       // n x 64 bytes
    uint32_t* best;
    uint32_t target[8];         // little-endian words, word 7 most significant
    uint32_t n;
    uint32_t pad;
};

// Batch SHA-256d (sha256d.hip). sha256d_batch: n messages of len bytes, stride bytes apart.
// sha256d_merkle_level: n output nodes from len 32-byte input nodes (stride unused).
// Mix-only batch header check (K4 + K6, sha256d.hip: kawpow_mixonly_batch), one lane per header:
// 120-byte KawPow headers in, 128-byte rows out = header hash | mix-only final | nBits boundary |
// claimed mix, all four in ProgPoW byte order (the boundary big-endian).
struct MixOnlyParams {
    const uint8_t* headers;
    uint8_t* out;      // n x 128 bytes
    uint32_t n;
    uint32_t stride;   // bytes between headers (>= 120)
};

// Batch DarkGravityWave v3 (dgw.hip): the expected nBits of every header of a linear batch from
// one (nTime, nBits) series = `a` ancestors of the batch (oldest first) then the n batch headers.
// out[i] = 0: header i is not a DGW header (BTC-retarget era): the host computes it.
struct DgwParams {
    const uint32_t* times;
    const uint32_t* bits;
    uint32_t* out;
    uint32_t a, n;
    int32_t base_height;           // height of the batch's parent
    int32_t dgw_activation_block;
    uint32_t kawpow_time, equihash_time;
    uint32_t pow_limit[8], kawpow_limit[8], equihash_limit[8];  // little-endian 32-bit limbs
    uint32_t pow_limit_compact, kawpow_limit_compact, equihash_limit_compact;
    uint32_t target_timespan;      // 180 x target spacing
};

struct Sha256dParams {
    const uint8_t* in;
    uint8_t* out;      // n x 32 bytes
    uint32_t len;
    uint32_t stride;
    uint32_t n;
    uint32_t pad;
};

// Device-resident batch header verification (header_batch.hip; models/verify.py).
struct HeaderBatchParams {
    const uint8_t* rows;       // n x 128: the packed batch (csrc/chain/headerbatch.hpp)
    const uint8_t* kinds;      // n: 0 KawPow, 2 Equihash, 3 pre-KawPow
    const uint8_t* mixonly;    // n x 128: kawpow_mixonly_batch rows
    struct KawpowVerifyJob* jobs;  // n
    uint32_t* job_program;     // n
    const uint32_t* full;      // n x 16: kawpow_verify_dag output (mix, final)
    uint8_t* out;              // n codes, then n x 32 block hashes (storage order)
    const uint32_t* eq_index;  // eq_n batch positions of the Equihash headers
    const uint32_t* eq_verdict;  // eq_n eq_verify verdicts
    const uint8_t* eq_hash;    // eq_n x 32 SHA256d of the serialized headers
    uint32_t n, eq_n;          // rows in the batch (the layout of `out`), Equihash headers given
    uint32_t first, count;     // the rows this launch covers: [first, first + count)
    uint32_t epoch_length;     // ethash epoch (7500 blocks; 2500 ProgPoW periods)
    int32_t last_checkpoint;   // KawPow headers at or below it get the mix-only check only (-1: none)
    uint8_t pow_limit[32];     // consensus powLimit, little-endian (CheckProofOfWork's target cap)
};

