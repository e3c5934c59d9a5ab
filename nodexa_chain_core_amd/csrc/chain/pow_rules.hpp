// Difficulty, proof-of-work and reward rules.
//
// Parity: DarkGravityWave v3 incl. the KawPow bootstrap and regtest
// min-difficulty rule (src/pow.cpp:18-102), BTC retarget (src/pow.cpp:104-180),
// GetNextWorkRequired dispatch on IsDGWActive (src/pow.cpp:140-155,
// src/validation.cpp:13512-13514), CheckProofOfWork (src/pow.cpp:182-199),
// GetBlockProof (src/chain.cpp:123-136), GetBlockSubsidy (Linux branch,
// src/validation.cpp:8988-8996), GetDifficulty (src/rpc/blockchain.cpp:56-81).
#pragma once

#include "params.hpp"

namespace nodexa {

// Minimal view of an indexed header (CBlockIndex subset used by consensus).
struct HeaderIndex {
    Uint256 hash;
    const HeaderIndex* prev = nullptr;
    int height = 0;
    u32 time = 0;
    u32 bits = 0;
    ArithU256 chain_work;
    BlockHeader header;
    const HeaderIndex* skip = nullptr;  // ancestor skip pointer
    int64_t median_time_past() const;
    const HeaderIndex* ancestor(int h) const;
};

constexpr int kDgwPastBlocks = 180;  // DGW window (src/pow.cpp:23)

u32 dark_gravity_wave(const HeaderIndex* last, const BlockHeader& next, const ChainParams& params);
// DGW's averaging + retarget over a chronological window of (nTime, nBits): element j is
// the last block, j-1, j-2, ... its ancestors (j >= 179). The caller has already handled
// the short-chain (height < 180) and regtest min-difficulty cases. Lets a linear header
// batch compute every header's expected nBits in parallel from the batch itself.
u32 dgw_average(const u32* times, const u32* bits, int64_t j, u32 next_time, const ChainParams& params);
u32 next_work_required_btc(const HeaderIndex* last, const BlockHeader& next, const ChainParams& params);
u32 calculate_next_work_required(const HeaderIndex* last, int64_t first_block_time, const ChainParams& params);
u32 next_work_required(const HeaderIndex* last, const BlockHeader& next, const ChainParams& params);
bool check_proof_of_work(const Uint256& hash, u32 bits, const ChainParams& params);
ArithU256 block_proof(u32 bits);
Amount block_subsidy(int height);
double difficulty_from_bits(u32 bits);

}  // namespace nodexa
