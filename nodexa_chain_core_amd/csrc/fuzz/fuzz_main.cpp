// libFuzzer harness for the native core (the reference's test_clore_fuzzy tier, SURVEY §4:
// src/test/test_clore_fuzzy.cpp deserializes 17 wire / disk types from AFL input).
//
// The first input byte picks the target, the rest is its input. Every target must either
// reject the bytes (an exception from the Reader or a false / error return) or accept them
// consistently: a block, header or transaction that parses with every byte consumed must
// re-serialize to exactly those bytes (the encodings are canonical, so anything else means a
// parse that dropped or invented data). Built with clang -fsanitize=fuzzer,address,undefined
// (_build.py fuzz); tests/test_fuzz.py runs it over a seed corpus for a fixed number of runs.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <stdexcept>
#include <string>

#include "../chain/assets.hpp"
#include "../chain/fees.hpp"
#include "../chain/indexes.hpp"
#include "../chain/interpreter.hpp"
#include "../chain/primitives.hpp"
#include "../crypto/secp256k1.hpp"
#include "../pow/legacy_algos.hpp"
#include "../pow/x16r.hpp"
#include "../store/bdb.hpp"

using namespace nodexa;

namespace {

[[noreturn]] void fail(const char* what) {
    std::fprintf(stderr, "fuzz invariant violated: %s\n", what);
    std::abort();
}

constexpr u32 kKawpowAlways = 0;            // every header in the 120-byte KawPow format
constexpr u32 kKawpowNever = 0xffffffffu;   // every header in the 80-byte legacy format

void fuzz_block(const Bytes& in, u32 act) {
    Reader r(in);
    Block b;
    try {
        b = Block::deserialize(r, act);
    } catch (const std::exception&) {
        return;
    }
    if (r.empty() && b.bytes(act) != in) fail("block re-serialization differs");
    bool mutated = false;
    (void)block_merkle_root(b, &mutated);
    (void)witness_commitment_index(b);
    for (const Transaction& tx : b.vtx) (void)check_transaction(tx);
}

void fuzz_header(const Bytes& in, u32 act) {
    Reader r(in);
    BlockHeader h;
    try {
        h = BlockHeader::deserialize(r, act);
    } catch (const std::exception&) {
        return;
    }
    if (r.empty() && h.bytes(act) != in) fail("header re-serialization differs");
    (void)h.kawpow_header_hash();
    if (h.is_equihash()) (void)h.equihash_input();
}

void fuzz_tx(const Bytes& in) {
    Reader r(in);
    Transaction tx;
    try {
        tx = Transaction::deserialize(r);
    } catch (const std::exception&) {
        return;
    }
    if (r.empty() && tx.bytes(true) != in) fail("transaction re-serialization differs");
    (void)check_transaction(tx);
    (void)tx.txid();
    (void)tx.wtxid();
}

void fuzz_script(const Bytes& in) {
    if (in.empty()) return;
    const u32 flags = in[0] & 1 ? kStandardScriptFlags : kMandatoryScriptFlags;
    const Bytes script(in.begin() + 1, in.end());
    std::vector<Bytes> stack;
    SigChecker none;
    ScriptError err{};
    (void)eval_script(stack, script, flags, none, in[0] & 2 ? SigVersion::WITNESS_V0 : SigVersion::BASE, &err);
    (void)is_valid_signature_encoding(script);
    (void)is_low_der_signature(script);
    (void)is_compressed_or_uncompressed_pubkey(script);
}

void fuzz_assets(const Bytes& in) {
    const std::string s(in.begin(), in.end());
    std::set<std::string> found;
    std::string err;
    (void)assets::check_verifier(s, found, err);
    try {
        std::map<std::string, bool> vals;
        for (const std::string& q : assets::verifier_qualifiers(assets::strip_verifier(s))) vals[q] = q.size() & 1;
        (void)assets::bool_expr(assets::strip_verifier(s), vals);
    } catch (const std::exception&) {
    }
    (void)assets::parent_name(s);
    assets::AssetOut out;
    (void)assets::parse_asset_out(in, out);
    std::string name, verifier;
    int flag = 0;
    u8 h160[20];
    (void)assets::parse_null_tag(in, name, flag, h160);
    (void)assets::parse_null_global(in, name, flag);
    (void)assets::parse_null_verifier(in, verifier);
}

void fuzz_snapshots(const Bytes& in, int which) {
    if (which == 0) {
        FeeEstimator f;
        std::string err;
        if (f.deserialize(in, &err)) {
            // a file that loads must write back in the same layout and load again
            FeeEstimator g;
            if (!g.deserialize(f.serialize(), &err)) fail("fee estimates do not reload");
            (void)f.estimate_smart_fee(6, true, nullptr, nullptr, nullptr);
        }
    } else if (which == 1) {
        assets::State st;
        if (st.deserialize(in)) {
            assets::State again;
            if (!again.deserialize(st.serialize())) fail("asset snapshot does not reload");
        }
    } else {
        ChainIndexes ix;
        (void)ix.deserialize(in);
    }
}

void fuzz_der(const Bytes& in) {
    secp::Scalar r, s;
    (void)secp::sig_parse_der_lax(in.data(), in.size(), r, s);
    if (in.size() >= 65) {
        u8 msg[32] = {0};
        (void)secp::verify_der(in.data(), 33, in.data() + 33, in.size() - 33, msg);
    }
}

}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
    if (size == 0) return 0;
    const Bytes in(data + 1, data + size);
    switch (data[0] % 15) {
    case 0: fuzz_block(in, kKawpowAlways); break;
    case 1: fuzz_block(in, kKawpowNever); break;
    case 2: fuzz_header(in, kKawpowAlways); break;
    case 3: fuzz_header(in, kKawpowNever); break;
    case 4: fuzz_tx(in); break;
    case 5: fuzz_script(in); break;
    case 6: fuzz_assets(in); break;
    case 7: fuzz_snapshots(in, 0); break;
    case 8: fuzz_snapshots(in, 1); break;
    case 9: fuzz_snapshots(in, 2); break;
    case 10: fuzz_der(in); break;
    case 11: {
        u8 prev[32] = {0}, out[32];
        if (in.size() >= 32) std::memcpy(prev, in.data(), 32);
        x16r_hash(in.data(), in.size(), prev, in.size() & 1, out);
        break;
    }
    case 12: {
        // HAVAL and GOST Streebog over the whole input; Lyra2 with small parameters taken from its
        // first bytes and the rest split into password and salt (inputs larger than the matrix
        // must be refused)
        if (in.size() < 8) break;
        (void)haval_hash(in.data() + 7, in.size() - 7, 3 + in[0] % 3, 128 + 32 * (in[1] % 5));
        (void)gost_streebog(in.data() + 7, in.size() - 7, in[1] & 1 ? 256 : 512);
        const size_t body = in.size() - 7, split = body ? in[6] % (body + 1) : 0;
        (void)lyra2_hash(in.data() + 7, split, in.data() + 7 + split, body - split, in[5], 1 + in[4] % 3,
                         u64(4) << (in[2] % 3), 1 + in[3] % 4, in[6] & 1);
        break;
    }
    case 13: {
        // a wallet.dat page walk (store/bdb.cpp): malformed pages must be refused, never read
        // past the buffer, and a tree with cycles must end; the sub-database is "main" or none
        try {
            (void)bdb::read_btree_bytes(std::string(in.begin(), in.end()), in.size() & 1 ? "main" : "");
        } catch (const std::runtime_error&) {
        }
        break;
    }
    case 14: {
        // the btree writer (wallet.dat export): records cut from the input (1-byte key length,
        // 2-byte value length) at a page size from the first byte, written and read back exactly
        bdb::Records recs;
        std::map<std::string, std::string> want;
        size_t at = 1;
        while (at + 3 <= in.size()) {
            const size_t kl = 1 + in[at] % 64, vl = (size_t(in[at + 1]) << 8 | in[at + 2]) % 6000;
            at += 3;
            if (at + kl + vl > in.size()) break;
            std::string k(reinterpret_cast<const char*>(in.data() + at), kl);
            std::string v(reinterpret_cast<const char*>(in.data() + at + kl), vl);
            at += kl + vl;
            if (want.emplace(k, v).second) recs.emplace_back(k, v);
        }
        if (in.empty()) break;
        const uint32_t ps = 512u << (in[0] % 4);  // 512 .. 4096
        const std::string file = bdb::write_btree_bytes(recs, "main", ps, std::string(20, '\x5a'));
        const bdb::Records back = bdb::read_btree_bytes(file, "main");
        if (back.size() != want.size()) __builtin_trap();
        size_t i = 0;
        for (const auto& kv : want) {
            if (back[i].first != kv.first || back[i].second != kv.second) __builtin_trap();
            ++i;
        }
        break;
    }
    }
    return 0;
}
