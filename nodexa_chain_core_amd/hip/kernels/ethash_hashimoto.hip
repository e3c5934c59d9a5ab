// Classic Ethash hashimoto over the resident DAG on gfx950 (SURVEY K-table "GPU classic
// hashimoto"; reference: src/crypto/ethash/lib/ethash/ethash.cpp:257-303 hash_seed / hash_mix /
// hash_final, 416-440 ethash::hash).
//
//   seed  = keccak512(header_hash || nonce_le)                  (64 bytes)
//   mix   = seed repeated to 32 words
//   64 x { p = fnv1(i ^ seed[0], mix[i % 32]) % pages ; mix = fnv1(mix, dataset page p) }
//   cmix  = 8 words, each fnv1-folded from 4 mix words;  final = keccak256(seed || cmix)
//
// Three launches on one stream: ethash_seed_batch (keccak512, one job per lane) -> ethash_mix_batch
// (the 64 page loads) -> ethash_final_batch (keccak256, one job per lane), seeds through an n x 64 B
// scratch. The mix kernel carries no keccak state, so it fits 8 waves per SIMD: the page loads are
// latency-bound dependent chains, and occupancy is what keeps the most of them in flight. In it,
// EH_HASHES hashes share a 16-lane DPP row (their loads in flight together); for each, lane l owns
// mix words 2l and 2l+1 and loads the matching 8 bytes of each 128-byte page, so a page is one
// contiguous 128-byte request per row; the loop is unrolled by 32 so the word that picks the next
// page (mix[i % 32]) is a compile-time lane, broadcast with one DPP row_newbcast. The DAG is the one
// KawPow searches (ops/ethash.DeviceEpoch): page p = 512-bit items 2p and 2p+1.
#include "kernel_params.h"
#include "keccak_device.hpp"

// hashes interleaved per 16-lane row of the mix kernel (their page loads in flight together):
// 2 measured best at epoch 384 (569 MH/s; 1: 505, 4: 563, 8: 563 -- profiles/README r5i)
#ifndef EH_HASHES
#define EH_HASHES 2
#endif

NX_DEV uint32_t eh_fnv1(uint32_t u, uint32_t v) { return (u * 0x01000193u) ^ v; }

NX_DEV uint32_t eh_fastmod(uint32_t x, const FastMod32& f) {
    const uint32_t t = __umulhi(x, f.m);
    const uint32_t q = (t + ((x - t) >> 1)) >> (f.s - 1);
    return x - q * f.d;
}

template <int J>
NX_DEV uint32_t eh_bcast(uint32_t x) {  // lane J of the 16-lane row, to every lane of the row
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + J, 0xf, 0xf, false);
}

// 16 accesses of H independent hashes with the mix word index base + 0..15 known at compile
// time: the H page loads of one access are in flight together.
template <int B, int H>
NX_DEV void eh_accesses(uint32_t i0, const uint32_t (&seed0)[H], uint32_t (&m0)[H], uint32_t (&m1)[H],
                        const uint2* __restrict__ dag, const FastMod32& pages, uint32_t lane) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int w = B + k;  // mix word i % 32
        uint2 d[H];
#pragma unroll
        for (int h = 0; h < H; ++h) {
            uint32_t v;
            switch (w >> 1) {  // compile-time after unrolling: one DPP broadcast
#define EH_CASE(L) case L: v = eh_bcast<L>((w & 1) ? m1[h] : m0[h]); break;
                EH_CASE(0) EH_CASE(1) EH_CASE(2) EH_CASE(3) EH_CASE(4) EH_CASE(5) EH_CASE(6) EH_CASE(7)
                EH_CASE(8) EH_CASE(9) EH_CASE(10) EH_CASE(11) EH_CASE(12) EH_CASE(13) EH_CASE(14)
                default: v = eh_bcast<15>((w & 1) ? m1[h] : m0[h]); break;
#undef EH_CASE
            }
            const uint32_t p = eh_fastmod(eh_fnv1((i0 + (uint32_t)k) ^ seed0[h], v), pages);
            d[h] = dag[(size_t)p * 16 + lane];
        }
#pragma unroll
        for (int h = 0; h < H; ++h) {
            m0[h] = eh_fnv1(m0[h], d[h].x);
            m1[h] = eh_fnv1(m1[h], d[h].y);
        }
    }
}

NX_DEV void eh_seed(const KawpowVerifyJob& jb, uint64_t seed[8]) {
    uint64_t a[25];
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = (uint64_t)jb.header[2 * k] | ((uint64_t)jb.header[2 * k + 1] << 32);
    a[4] = jb.nonce;
    a[5] = 0x01ULL;  // Keccak padding of a 40-byte message (rate 72)
#pragma unroll
    for (int k = 6; k < 25; ++k) a[k] = 0;
    a[8] = 0x8000000000000000ULL;
    keccak_f1600(a);
#pragma unroll
    for (int k = 0; k < 8; ++k) seed[k] = a[k];
}

// Phase 1: seed = keccak512(header || nonce), one job per lane, into the seed scratch (n x 64 B).
extern "C" __global__ __launch_bounds__(256) void ethash_seed_batch(EthashHashParams p) {
    const uint32_t job = blockIdx.x * blockDim.x + threadIdx.x;
    if (job >= p.num_jobs) return;
    uint64_t seed[8];
    if (p.jobs != nullptr) {
        eh_seed(p.jobs[job], seed);
    } else {  // search mode: one header, consecutive nonces
        KawpowVerifyJob jb;
#pragma unroll
        for (int k = 0; k < 8; ++k) jb.header[k] = p.header[k];
        jb.nonce = p.start_nonce + job;
        eh_seed(jb, seed);
    }
    uint4* o = (uint4*)(p.seeds + (size_t)job * 16);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        o[k] = make_uint4((uint32_t)seed[2 * k], (uint32_t)(seed[2 * k] >> 32), (uint32_t)seed[2 * k + 1],
                          (uint32_t)(seed[2 * k + 1] >> 32));
}

// Phase 2: the 64 dependent page loads, H hashes per 16-lane row; the row's 32 mix words fold into
// cmix (8 words), written to the job's mix slot of `out`. Without a keccak state the kernel stays
// under 64 VGPRs: 8 waves per SIMD keep the most page loads in flight.
template <int H>
NX_DEV void eh_mix(const EthashHashParams& p) {
    const uint32_t lane = threadIdx.x & 15u;
    const uint32_t first = (blockIdx.x * (blockDim.x / 16u) + threadIdx.x / 16u) * (uint32_t)H;
    if (first >= p.num_jobs) return;  // whole rows only: the DPP broadcasts never reach an exited lane
    uint32_t seed0[H], m0[H], m1[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
        // a row past the batch end repeats its last valid job (written once, by the slot owning it)
        const uint32_t* sd = p.seeds + (size_t)min(first + (uint32_t)h, p.num_jobs - 1u) * 16;
        // mix word w = seed word w % 16: lane l holds words 2l, 2l+1 = seed words 2(l%8), 2(l%8)+1
        const uint2 s = *(const uint2*)(sd + 2 * (lane & 7u));
        m0[h] = s.x;
        m1[h] = s.y;
        seed0[h] = sd[0];
    }
    const uint2* __restrict__ dag = (const uint2*)p.dag;
#pragma unroll 1
    for (uint32_t i = 0; i < 64; i += 32) {
        eh_accesses<0, H>(i, seed0, m0, m1, dag, p.pages, lane);
        eh_accesses<16, H>(i + 16, seed0, m0, m1, dag, p.pages, lane);
    }
#pragma unroll
    for (int h = 0; h < H; ++h) {
        // cmix[k] = fnv1(fnv1(fnv1(mix[4k], mix[4k+1]), mix[4k+2]), mix[4k+3]): lanes 2k and 2k+1;
        // each lane folds its own pair, then even lanes take the odd neighbour's pair
        const uint32_t x0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)m0[h], 0x101, 0xf, 0xf, false);  // row_shl:1
        const uint32_t x1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)m1[h], 0x101, 0xf, 0xf, false);
        const uint32_t c = eh_fnv1(eh_fnv1(eh_fnv1(m0[h], m1[h]), x0), x1);  // valid on even lanes
        if (first + (uint32_t)h < p.num_jobs && (lane & 1u) == 0)
            p.out[(size_t)(first + h) * 16 + lane / 2] = c;
    }
}

// Phase 3: final = keccak256(seed || cmix), one job per lane.
extern "C" __global__ __launch_bounds__(256) void ethash_final_batch(EthashHashParams p) {
    const uint32_t job = blockIdx.x * blockDim.x + threadIdx.x;
    if (job >= p.num_jobs) return;
    const uint4* sd = (const uint4*)(p.seeds + (size_t)job * 16);
    const uint4* cm = (const uint4*)(p.out + (size_t)job * 16);
    uint64_t a[25];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint4 v = sd[k];
        a[2 * k] = (uint64_t)v.x | ((uint64_t)v.y << 32);
        a[2 * k + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint4 v = cm[k];
        a[8 + 2 * k] = (uint64_t)v.x | ((uint64_t)v.y << 32);
        a[9 + 2 * k] = (uint64_t)v.z | ((uint64_t)v.w << 32);
    }
    a[12] = 0x01ULL;  // 96-byte message, rate 136
#pragma unroll
    for (int k = 13; k < 25; ++k) a[k] = 0;
    a[16] = 0x8000000000000000ULL;
    keccak_f1600(a);
    uint4* o = (uint4*)(p.out + (size_t)job * 16 + 8);
    o[0] = make_uint4((uint32_t)a[0], (uint32_t)(a[0] >> 32), (uint32_t)a[1], (uint32_t)(a[1] >> 32));
    o[1] = make_uint4((uint32_t)a[2], (uint32_t)(a[2] >> 32), (uint32_t)a[3], (uint32_t)(a[3] >> 32));
    if (p.hits != nullptr) {
        // final <= boundary as 256-bit big-endian numbers (ethash::is_less_or_equal): byte-swapped
        // words compared from the most significant one
        bool le = true, decided = false;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t w = (uint32_t)(a[k / 2] >> (32 * (k & 1)));
            const uint32_t f = __builtin_bswap32(w), b = __builtin_bswap32(p.boundary[k]);
            if (!decided && f != b) {
                le = f < b;
                decided = true;
            }
        }
        if (le) {
            const uint32_t slot = atomicAdd(p.hits, 1u);
            if (slot < p.max_hits) p.hits[1 + slot] = job;
        }
    }
}

extern "C" __global__ __launch_bounds__(256, 8) void ethash_mix_batch(EthashHashParams p) { eh_mix<EH_HASHES>(p); }
