// Block-level consensus checks (the structural subset the PoW engine owns).
//
// Parity: CheckBlock (src/validation.cpp:11667: merkle root + mutation,
// size/weight limits, coinbase placement, duplicate txids), ContextualCheck-
// Block (:11877: BIP34 coinbase height, witness commitment), and the CLORE
// reward rules in ConnectBlock (:10405-10440: coinbase value <= subsidy+fees,
// vout[1] == subsidy*pct/100 paid to the community-autonomous script).
// Script/UTXO validation (fees of non-coinbase transactions) stays out of
// scope (DEFER); callers pass the fees they know.
#pragma once

#include "headerchain.hpp"

namespace nodexa {

constexpr size_t kMaxBlockWeight = 8000000;  // after HIP2 (src/consensus/consensus.h:14-22)
constexpr size_t kWitnessScaleFactor = 4;
constexpr size_t kMinTransactionWeight = kWitnessScaleFactor * 60;

struct BlockCheck {
    bool ok = false;
    std::string reject;
    int dos = 0;
};

BlockCheck check_block(const Block& b, const ChainParams& p, bool check_merkle = true,
                       const assets::Flags& asset_flags = assets::Flags{});
BlockCheck contextual_check_block(const Block& b, const ChainParams& p, int height);
BlockCheck check_coinbase_rewards(const Block& b, const ChainParams& p, int height, Amount fees,
                                  bool fees_known);
// BIP34 coinbase scriptSig prefix for `height` (CScript() << nHeight).
Bytes coinbase_height_prefix(int height);

}  // namespace nodexa
