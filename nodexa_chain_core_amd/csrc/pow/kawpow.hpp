// KawPow = ProgPoW 0.9.4 with Ravencoin/Clore "RAVENCOINKAWPOW" keccak padding.
//
// Parity (behaviour; see SURVEY.md Appendix A for the bit-level spec):
//   constants         src/crypto/ethash/include/ethash/progpow.hpp:19-27
//   program RNG       src/crypto/ethash/lib/ethash/progpow.cpp:46-88
//   random_math/merge src/crypto/ethash/lib/ethash/progpow.cpp:91-144
//   round / init_mix  src/crypto/ethash/lib/ethash/progpow.cpp:179-263
//   hash_mix / reduce src/crypto/ethash/lib/ethash/progpow.cpp:265-295
//   hash/verify/...   src/crypto/ethash/lib/ethash/progpow.cpp:298-579
//
// Design: the per-period program is *materialised* once (KawpowProgram) instead
// of re-running the KISS99 stream inside every round. The same object drives
// the CPU golden model here and the gfx950 code generator
// (kawpow_codegen.cpp), so both share one definition of the instruction
// stream; the golden vectors pin it.
#pragma once

#include "ethash.hpp"

namespace nodexa {

constexpr int kPeriodLength = 3;
constexpr int kNumRegs = 32;
constexpr int kNumLanes = 16;
constexpr int kNumCacheAccesses = 11;
constexpr int kNumMathOps = 18;
constexpr int kDagLoads = 4;  // words per lane per round
constexpr int kNumRounds = 64;

struct Kiss99 {
    u32 z, w, jsr, jcong;
    inline u32 operator()() {
        z = 36969 * (z & 0xffff) + (z >> 16);
        w = 18000 * (w & 0xffff) + (w >> 16);
        jcong = 69069 * jcong + 1234567;
        jsr ^= (jsr << 17);
        jsr ^= (jsr >> 13);
        jsr ^= (jsr << 5);
        return (((z << 16) + w) ^ jcong) + jsr;
    }
};

struct KawpowProgram {
    u64 period = ~0ULL;  // sentinel: not yet generated
    struct CacheOp { u8 src, dst; u32 sel; };
    struct MathOp { u8 src1, src2, dst; u32 sel1, sel2; };
    CacheOp cache[kNumCacheAccesses];
    MathOp math[kNumMathOps];
    u8 dag_dst[kDagLoads];
    u32 dag_sel[kDagLoads];
};

KawpowProgram make_kawpow_program(u64 period);
inline u64 kawpow_period(int block_number) { return u64(block_number / kPeriodLength); }

inline u32 kawpow_math(u32 a, u32 b, u32 sel) {
    switch (sel % 11) {
        default:
        case 0: return a + b;
        case 1: return a * b;
        case 2: return mulhi32(a, b);
        case 3: return a < b ? a : b;
        case 4: return rotl32(a, b);
        case 5: return rotr32(a, b);
        case 6: return a & b;
        case 7: return a | b;
        case 8: return a ^ b;
        case 9: return clz32(a) + clz32(b);
        case 10: return popc32(a) + popc32(b);
    }
}

inline void kawpow_merge(u32& a, u32 b, u32 sel) {
    const u32 x = ((sel >> 16) % 31) + 1;
    switch (sel % 4) {
        case 0: a = (a * 33) + b; break;
        case 1: a = (a ^ b) * 33; break;
        case 2: a = rotl32(a, x) ^ b; break;
        case 3: a = rotr32(a, x) ^ b; break;
    }
}

struct KawpowResult {
    Hash256 final_hash;
    Hash256 mix_hash;
};

// Light-mode hash (DAG items computed from the light cache on demand).
KawpowResult kawpow_hash(const EpochContext& ctx, int block_number, const Hash256& header_hash,
                         u64 nonce);
// Full-DAG hash (HostDag filled lazily).
KawpowResult kawpow_hash_full(HostDag& dag, int block_number, const Hash256& header_hash, u64 nonce);
bool kawpow_verify(const EpochContext& ctx, int block_number, const Hash256& header_hash,
                   const Hash256& mix_hash, u64 nonce, const Hash256& boundary);
// "mix-only" final hash trusting the supplied mix (progpow::hash_no_verify).
Hash256 kawpow_hash_no_verify(int block_number, const Hash256& header_hash, const Hash256& mix_hash,
                              u64 nonce);
// Seed (state2[0..7]) of the initial keccak-f800 absorb.
void kawpow_initial_state(const Hash256& header_hash, u64 nonce, u32 state2[8]);
Hash256 kawpow_final(const u32 state2[8], const Hash256& mix_hash);

struct KawpowSearchResult {
    bool found = false;
    u64 nonce = 0;
    KawpowResult result;
};
// First nonce in [start, start+iterations) with final <= boundary.
KawpowSearchResult kawpow_search_light(const EpochContext& ctx, int block_number,
                                       const Hash256& header_hash, const Hash256& boundary,
                                       u64 start_nonce, u64 iterations);
KawpowSearchResult kawpow_search_full(HostDag& dag, int block_number, const Hash256& header_hash,
                                      const Hash256& boundary, u64 start_nonce, u64 iterations,
                                      int threads);
// Count of hashes evaluated per second on the host (full DAG, `threads`).
double kawpow_cpu_hashrate(HostDag& dag, int block_number, u64 nonces, int threads);

// gfx950 HIP source for one period (see hip/kernels/kawpow_search.hip).
std::string kawpow_codegen_hip(const KawpowProgram& prog);
// 64-word data encoding of a period's program for the batch-verify kernel
// (hip/kernels/kawpow_verify.hip, layout documented there).
std::vector<u32> kawpow_program_words(const KawpowProgram& prog);

}  // namespace nodexa
