#include "params.hpp"

#include <stdexcept>
#include <vector>

#include "script.hpp"

namespace nodexa {

Block make_genesis_block(const std::string& timestamp, const Bytes& output_script, u32 time, u32 nonce, u32 bits,
                         int32_t version, Amount reward) {
    Transaction tx;
    tx.version = 1;
    tx.vin.resize(1);
    tx.vout.resize(1);
    ScriptBuilder sig;
    sig.push_num(0).push_int(486604799).push_num(4).push_data(Bytes(timestamp.begin(), timestamp.end()));
    tx.vin[0].script_sig = sig.s;
    tx.vout[0].value = reward;
    tx.vout[0].script_pubkey = output_script;
    Block g;
    g.header.time = time;
    g.header.bits = bits;
    g.header.nonce = nonce;
    g.header.version = version;
    g.vtx.push_back(tx);
    g.header.merkle_root = block_merkle_root(g);
    return g;
}

namespace {

Block clore_genesis(u32 time, u32 nonce, u32 bits, int32_t version, Amount reward) {
    const std::string ts = "The Times 03/30/2021 Bitcoin is name of the game for new generation of firms";
    ScriptBuilder out;
    out.push_data(hex_decode(
        "04678afdb0fe5548271967f1a67130b7105cd6a828e03909a67962e0ea1f61deb649f6bc3f4cef38c4f35504e51ec112de5c384df7ba0b8d578a4c702b6bf11d5f"));
    out.op(OP_CHECKSIG);
    return make_genesis_block(ts, out.s, time, nonce, bits, version, reward);
}

}  // namespace

namespace {

// test and regtest share one set of burn addresses (src/chainparams.cpp:393-403, 538-548)
const std::vector<std::string> kTestBurnAddresses = {
    "J1VQJKLSLVZ4syiCAx5hEPq8BrkFaxAXAi", "J2yh4DiLETuVVDvpvBNSq3QCmHcdMmNEdp", "J3PE3FsHqfszvz7nhwK2Gc32wykrc7pNMA",
    "J4yKRTYF2nRryYEnupsNnQQmRKsQhdspYB", "J58ndjHjLYKHMszr4ehUg9YMWPAiXNEepa", "J68wpmVvdE6bMSkiCEDQWCHCKZs4VVdE2G",
    "J7MSidYgNJrPE15ouEsXPYXFYH2AAPXmhr", "J8uX8jfZn14P1VNzh6YjSzLaRTQAdoFSHn", "J9CrKy8m548AvSbcv1mcn7tyJQkgcwVfj6",
    "JGYQBki6wWWnJLp2dcgdtNZWs9a2e1nXM3"};

void set_burn_addresses(ChainParams& p, const std::vector<std::string>& a) {
    Bytes* spk[10] = {&p.assets.spk_root, &p.assets.spk_reissue, &p.assets.spk_sub, &p.assets.spk_unique,
                      &p.assets.spk_msgchannel, &p.assets.spk_qualifier, &p.assets.spk_subqualifier,
                      &p.assets.spk_restricted, &p.assets.spk_tag, &p.assets.spk_global};
    for (int i = 0; i < 10; ++i) {
        p.asset_burn_addresses[i] = a[size_t(i)];
        if (!address_to_script(a[size_t(i)], p.pubkey_prefix, p.script_prefix, *spk[i]))
            throw std::logic_error("bad burn address " + a[size_t(i)]);
    }
}

}  // namespace

ChainParams make_chain_params(const std::string& network) {
    ChainParams p;
    if (network == "main") {
        p.network_id = "main";
        p.consensus.pow_limit = Uint256::from_hex("00ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff");
        p.consensus.kawpow_limit = p.consensus.pow_limit;
        p.message_start[0] = 0x41; p.message_start[1] = 0x49; p.message_start[2] = 0x41; p.message_start[3] = 0x49;
        p.default_port = 8788;
        p.default_rpc_port = 9766;
        p.pubkey_prefix = 23;
        p.script_prefix = 122;
        p.genesis = clore_genesis(1651442858, 3244753, 0x1e00ffff, 4, 5000 * COIN);
        p.consensus.genesis_hash = Uint256::from_hex("0000000a50fdaaf22f1c98b8c61559e15ab2269249aa1fb20683180703cdbf07");
        p.checkpoints[0] = p.consensus.genesis_hash;
        p.checkpoints[2] = Uint256::from_hex("003714ec51ec4bd78e1b548bf1c198711ef973d248b6bef7b5fd17a091e27e6f");
        p.checkpoints[3960] = Uint256::from_hex("00000000fa933b399211df8adc614d69ab0fd7ed4cce194e1fce0f7045fcc8db");
        p.community_autonomous_pct = 50;
        p.community_autonomous_address = "AePr762UcuQrGoa3TRQpGMX6byRjuXw97A";
        p.dgw_activation_block = 1;
        p.kawpow_activation_time = 1651444217;
        p.x16rv2_activation_time = 1569945600;
        set_burn_addresses(p, {"AP6RNAdjGgkX2QERU3Gr5VV5hvidu6xgau", "AKsyQ9K9Kxftcb77Veiv91kA2VugPY45PL",
                               "AbXjGsYEt89DUARDsQoXLAB3t4EpKUd1D8", "APZ5XSUwfKXDtscpoPbWfNkeiNu3FFu6ee",
                               "AVPHkMz1GCxqE85ZuoxsBWY62Fi1ygyBnG", "AXEv5tmqu6cnaskJbmrEEPKQGTnCkWBBTk",
                               "AM2okBkzJb21QyMGepGqmintGNnCJuVoQs", "AMR2ckKABVwQnhdFaQiQaqfoqAQLSZdV2T",
                               "AcjqNXmzBpoBCGgfzSMJqwZLnYiF4zoqtL", "AZuJi37imwSjTFBwExtJ12tG1BvSnUctZg"});
    } else if (network == "test") {
        p.network_id = "test";
        p.consensus.pow_limit = Uint256::from_hex("00ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff");
        p.consensus.kawpow_limit = p.consensus.pow_limit;
        p.message_start[0] = 0x60; p.message_start[1] = 0x63; p.message_start[2] = 0x56; p.message_start[3] = 0x65;
        p.default_port = 4568;
        p.default_rpc_port = 19766;
        p.pubkey_prefix = 42;
        p.script_prefix = 124;
        p.genesis = clore_genesis(1670019499, 11903232, 0x1e00ffff, 4, 5000 * COIN);
        p.community_autonomous_pct = 15;
        p.community_autonomous_address = "J8db9nuaVL3Jo8hDcfKh77pZnG2J8jvxWH";
        p.dgw_activation_block = 1;
        p.kawpow_activation_time = 1653247613;
        p.x16rv2_activation_time = 1567533600;
        p.assets.testnet = true;
        set_burn_addresses(p, kTestBurnAddresses);
    } else if (network == "regtest") {
        p.network_id = "regtest";
        p.consensus.subsidy_halving_interval = 150;
        p.consensus.pow_limit = Uint256::from_hex("7fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff");
        p.consensus.kawpow_limit = p.consensus.pow_limit;
        p.consensus.pow_allow_min_difficulty_blocks = true;
        p.consensus.pow_no_retargeting = true;
        p.message_start[0] = 0x44; p.message_start[1] = 0x52; p.message_start[2] = 0x4F; p.message_start[3] = 0x57;
        p.default_port = 19444;
        p.default_rpc_port = 19443;
        p.pubkey_prefix = 42;
        p.script_prefix = 124;
        p.genesis = clore_genesis(1524179366, 1, 0x207fffff, 4, 5000 * COIN);
        // The reference asserts 0b2c703d.. / merkle 28ff00a8.. here
        // (src/chainparams.cpp:494-495) — Ravencoin's values, inconsistent with
        // the Clore coinbase it actually builds (merkle 7c1d7173.., identical to
        // mainnet). We keep what the construction yields: the X16R hash of this
        // header, computed by HeaderChain (genesis_hash left null here).
        p.community_autonomous_pct = 10;
        p.community_autonomous_address = "JCPncGFawSDgP3CmG19MB6cbKP5XuhXY4u";
        p.dgw_activation_block = 200;
        p.kawpow_activation_time = 3582830167u;
        p.x16rv2_activation_time = 1569931200;
        p.mine_blocks_on_demand = true;
        p.mining_requires_peers = false;
        set_burn_addresses(p, kTestBurnAddresses);
    } else {
        throw std::invalid_argument("unknown chain " + network);
    }
    return p;
}

}  // namespace nodexa
