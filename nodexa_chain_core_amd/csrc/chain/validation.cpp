#include "validation.hpp"

#include <algorithm>
#include <set>

#include "../crypto/sha256.hpp"
#include "interpreter.hpp"
#include "script.hpp"

namespace nodexa {

namespace {
BlockCheck fail(const char* reason, int dos = 100) {
    BlockCheck c;
    c.reject = reason;
    c.dos = dos;
    return c;
}
BlockCheck pass() {
    BlockCheck c;
    c.ok = true;
    return c;
}
}  // namespace

Bytes coinbase_height_prefix(int height) { return ScriptBuilder().push_int(height).s; }

BlockCheck check_block(const Block& b, const ChainParams& p, bool check_merkle, const assets::Flags& asset_flags) {
    if (check_merkle) {
        bool mutated = false;
        const Uint256 root = block_merkle_root(b, &mutated);
        if (root != b.header.merkle_root) return fail("bad-txnmrklroot");
        if (mutated) return fail("bad-txns-duplicate");
    }
    if (b.vtx.empty() || b.vtx.size() * kMinTransactionWeight > kMaxBlockWeight ||
        b.stripped_size(p.kawpow_activation_time) * kWitnessScaleFactor > kMaxBlockWeight)
        return fail("bad-blk-length");
    if (!b.vtx[0].is_coinbase()) return fail("bad-cb-missing");
    for (size_t i = 1; i < b.vtx.size(); ++i)
        if (b.vtx[i].is_coinbase()) return fail("bad-cb-multiple");
    const size_t sig = b.vtx[0].vin[0].script_sig.size();
    if (sig < 2 || sig > 100) return fail("bad-cb-length");
    // CheckTransaction on every transaction, with the asset rules (src/validation.cpp CheckBlock)
    for (auto& tx : b.vtx) {
        const std::string why = check_transaction(tx, true, &p.assets, &asset_flags, true, false);
        if (!why.empty()) {
            BlockCheck c;
            c.reject = why;
            c.dos = (why == "bad-txns-vin-empty" || why == "bad-txns-vout-empty" || why == "bad-txns-prevout-null") ? 10 : 100;
            if (why == "bad-txns-coinbase-contains-asset-txes" || why == "bad-txns-asset-reissued-amount-isn't-zero") c.dos = 0;
            return c;
        }
    }
    return pass();
}

BlockCheck contextual_check_block(const Block& b, const ChainParams& p, int height) {
    // BIP34: coinbase scriptSig starts with the serialized height
    const Bytes expect = coinbase_height_prefix(height);
    const Bytes& sig = b.vtx[0].vin[0].script_sig;
    if (sig.size() < expect.size() || !std::equal(expect.begin(), expect.end(), sig.begin()))
        return fail("bad-cb-height");
    // witness commitment
    bool have_witness = false;
    const int commitpos = witness_commitment_index(b);
    if (p.consensus.segwit_enabled && commitpos != -1) {
        const auto& wit = b.vtx[0].vin[0].witness;
        if (wit.size() != 1 || wit[0].size() != 32) return fail("bad-witness-nonce-size");
        Uint256 root = block_witness_merkle_root(b);
        u8 buf[64], commit[32];
        std::memcpy(buf, root.data, 32);
        std::memcpy(buf + 32, wit[0].data(), 32);
        sha256d(buf, 64, commit);
        const Bytes& spk = b.vtx[0].vout[size_t(commitpos)].script_pubkey;
        if (std::memcmp(commit, spk.data() + 6, 32) != 0) return fail("bad-witness-merkle-match");
        have_witness = true;
    }
    if (!have_witness)
        for (auto& tx : b.vtx)
            if (tx.has_witness()) return fail("unexpected-witness");
    if (b.weight(p.kawpow_activation_time) > kMaxBlockWeight) return fail("bad-blk-weight");
    return pass();
}

BlockCheck check_coinbase_rewards(const Block& b, const ChainParams& p, int height, Amount fees, bool fees_known) {
    const Amount subsidy = block_subsidy(height);
    if (fees_known && b.vtx[0].value_out() > subsidy + fees) return fail("bad-cb-amount");
    if (b.vtx[0].vout.size() < 2) return fail("bad-cb-community-autonomous-amount");
    const Amount community = subsidy * p.community_autonomous_pct / 100;
    if (b.vtx[0].vout[1].value != community) return fail("bad-cb-community-autonomous-amount");
    Bytes script;
    if (!address_to_script(p.community_autonomous_address, p.pubkey_prefix, p.script_prefix, script))
        return fail("bad-community-address-param", 0);
    if (b.vtx[0].vout[1].script_pubkey != script) return fail("bad-cb-community-autonomous-address");
    return pass();
}

}  // namespace nodexa
