// Chain parameters for main / test / regtest.
//
// Parity: CMainParams / CTestNetParams / CRegTestParams
// (src/chainparams.cpp:106-573), Consensus::Params (src/consensus/params.h:49-82),
// X16RV2 activation times (src/primitives/block.cpp:15-17), genesis
// construction (src/chainparams.cpp:17-60).
//
// New (not in the reference): `kawpow_activation_time` is overridable per
// process (-kawpowactivationtime, needed to exercise KawPow on regtest,
// SURVEY §0.6), and the Equihash(200,9) header extension has its own
// activation that is disabled (UINT32_MAX) on every reference network.
#pragma once

#include <map>

#include "assets.hpp"
#include "primitives.hpp"

namespace nodexa {

struct ConsensusParams {
    Uint256 genesis_hash;
    int subsidy_halving_interval = 2100000;
    Uint256 pow_limit;
    Uint256 kawpow_limit;
    // Equihash-era bootstrap target (DGW returns it until 180 Equihash blocks
    // fill the window, mirroring the KawPow switch rule); null = pow_limit.
    Uint256 equihash_limit;
    int64_t pow_target_spacing = 60;
    int64_t pow_target_timespan = 2016 * 60;
    bool pow_allow_min_difficulty_blocks = false;
    bool pow_no_retargeting = false;
    bool segwit_enabled = true;
    int64_t difficulty_adjustment_interval() const { return pow_target_timespan / pow_target_spacing; }
};

struct ChainParams {
    std::string network_id;  // "main" | "test" | "regtest"
    ConsensusParams consensus;
    u8 message_start[4] = {0, 0, 0, 0};
    int default_port = 0;
    int default_rpc_port = 0;
    u8 pubkey_prefix = 0;
    u8 script_prefix = 0;
    Block genesis;
    std::map<int, Uint256> checkpoints;
    int community_autonomous_pct = 0;
    std::string community_autonomous_address;
    int dgw_activation_block = 1;
    int max_reorg_depth = 60;
    int min_reorg_peers = 4;
    int64_t min_reorg_age = 60 * 60 * 12;
    u32 kawpow_activation_time = 0;
    u32 x16rv2_activation_time = 0;
    bool mine_blocks_on_demand = false;
    bool mining_requires_peers = true;
    // Equihash(200,9) extension (new, off on reference networks).
    u32 equihash_activation_time = 0xffffffffu;
    int equihash_n = 200;
    int equihash_k = 9;
    // Asset layer: burn amounts and burn scripts (src/chainparams.cpp burn addresses).
    assets::Params assets;
    std::string asset_burn_addresses[10];  // root, reissue, sub, unique, msgchannel, qualifier, subqualifier,
                                           // restricted, tag, global

    PowAlgo algo_for(u32 time) const {
        if (time >= kawpow_activation_time) return PowAlgo::KAWPOW;
        return time >= x16rv2_activation_time ? PowAlgo::X16RV2 : PowAlgo::X16R;
    }
    // Last checkpoint height (or -1) — governs mix-only vs full KawPow checks.
    int last_checkpoint_height() const { return checkpoints.empty() ? -1 : checkpoints.rbegin()->first; }
};

// Builds fresh params for a network ("main", "test", "regtest").
ChainParams make_chain_params(const std::string& network);
// Genesis block exactly as CreateGenesisBlock builds it.
Block make_genesis_block(const std::string& timestamp, const Bytes& output_script, u32 time, u32 nonce, u32 bits,
                         int32_t version, Amount reward);

}  // namespace nodexa
