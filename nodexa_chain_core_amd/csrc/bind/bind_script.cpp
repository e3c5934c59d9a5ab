// Bindings for secp256k1 (crypto/secp256k1.*) and the script interpreter (chain/interpreter.*).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <set>

#include "../chain/coins.hpp"
#include "../chain/indexes.hpp"
#include "../chain/interpreter.hpp"
#include "../chain/sigcache.hpp"
#include "../chain/params.hpp"
#include "../crypto/secp256k1.hpp"
#include "../crypto/secp256k1_model32.hpp"

namespace py = pybind11;
using namespace nodexa;

PYBIND11_MAKE_OPAQUE(std::vector<PendingSig>)

namespace {

Bytes bytes_of(const py::bytes& b) {
    std::string s = b;
    return Bytes(s.begin(), s.end());
}
py::bytes pyb(const u8* p, size_t n) { return py::bytes(reinterpret_cast<const char*>(p), n); }
py::bytes pyb(const Bytes& b) { return pyb(b.data(), b.size()); }

void need32(const std::string& s, const char* what) {
    if (s.size() != 32) throw std::invalid_argument(std::string(what) + " must be 32 bytes");
}

Transaction tx_of(const py::bytes& raw) {
    const Bytes b = bytes_of(raw);
    Reader r(b);
    Transaction tx = Transaction::deserialize(r, true);
    if (!r.empty()) throw std::invalid_argument("trailing bytes after transaction");
    return tx;
}

std::vector<Bytes> stack_of(const std::vector<py::bytes>& v) {
    std::vector<Bytes> out;
    out.reserve(v.size());
    for (auto& x : v) out.push_back(bytes_of(x));
    return out;
}

}  // namespace

void bind_script(py::module_& m) {
    // ---------------------------------------------------------------- secp256k1
    m.def("secp_pubkey_create", [](const py::bytes& key, bool compressed) -> py::object {
        const std::string k = key;
        need32(k, "key");
        secp::Ge p;
        if (!secp::pubkey_create(reinterpret_cast<const u8*>(k.data()), p)) return py::none();
        u8 out[65];
        return pyb(out, secp::pubkey_serialize(p, compressed, out));
    }, py::arg("key"), py::arg("compressed") = true, "public key of a 32-byte secret (None if invalid)");
    m.def("secp_pubkey_normalize", [](const py::bytes& pub, bool compressed) -> py::object {
        const std::string s = pub;
        secp::Ge p;
        if (!secp::pubkey_parse(reinterpret_cast<const u8*>(s.data()), s.size(), p)) return py::none();
        u8 out[65];
        return pyb(out, secp::pubkey_serialize(p, compressed, out));
    }, py::arg("pubkey"), py::arg("compressed") = true, "parse (02/03/04/06/07) and re-serialize, None if invalid");
    m.def("secp_sign", [](const py::bytes& msg, const py::bytes& key) -> py::object {
        const std::string m32 = msg, k = key;
        need32(m32, "msg");
        need32(k, "key");
        secp::Scalar r, s;
        if (!secp::ecdsa_sign(reinterpret_cast<const u8*>(m32.data()), reinterpret_cast<const u8*>(k.data()), r, s))
            return py::none();
        u8 der[72];
        return pyb(der, secp::sig_serialize_der(r, s, der));
    }, "RFC 6979 low-S DER signature (CKey::Sign with test_case 0)");
    m.def("secp_verify", [](const py::bytes& pub, const py::bytes& sig, const py::bytes& msg) {
        const std::string p = pub, sg = sig, m32 = msg;
        need32(m32, "msg");
        return secp::verify_der(reinterpret_cast<const u8*>(p.data()), p.size(), reinterpret_cast<const u8*>(sg.data()),
                                sg.size(), reinterpret_cast<const u8*>(m32.data()));
    }, "CPubKey::Verify: lax DER, S normalised");
    m.def("secp_sign_compact", [](const py::bytes& msg, const py::bytes& key, bool compressed) -> py::object {
        const std::string m32 = msg, k = key;
        need32(m32, "msg");
        need32(k, "key");
        u8 out[65];
        if (!secp::sign_compact(reinterpret_cast<const u8*>(m32.data()), reinterpret_cast<const u8*>(k.data()),
                                compressed, out))
            return py::none();
        return pyb(out, 65);
    });
    m.def("secp_recover_compact", [](const py::bytes& msg, const py::bytes& sig) -> py::object {
        const std::string m32 = msg, s = sig;
        need32(m32, "msg");
        if (s.size() != 65) return py::none();
        secp::Ge p;
        bool compressed = false;
        if (!secp::recover_compact(reinterpret_cast<const u8*>(m32.data()), reinterpret_cast<const u8*>(s.data()), p,
                                   compressed))
            return py::none();
        u8 out[65];
        return pyb(out, secp::pubkey_serialize(p, compressed, out));
    });
    m.def("secp_seckey_tweak_add", [](const py::bytes& key, const py::bytes& tweak) -> py::object {
        std::string k = key;
        const std::string t = tweak;
        need32(k, "key");
        need32(t, "tweak");
        if (!secp::seckey_tweak_add(reinterpret_cast<u8*>(k.data()), reinterpret_cast<const u8*>(t.data())))
            return py::none();
        return py::bytes(k);
    });
    m.def("secp_pubkey_tweak_add", [](const py::bytes& pub, const py::bytes& tweak) -> py::object {
        const std::string p = pub, t = tweak;
        need32(t, "tweak");
        secp::Ge g;
        if (!secp::pubkey_parse(reinterpret_cast<const u8*>(p.data()), p.size(), g)) return py::none();
        if (!secp::pubkey_tweak_add(g, reinterpret_cast<const u8*>(t.data()))) return py::none();
        u8 out[65];
        return pyb(out, secp::pubkey_serialize(g, p.size() == 33, out));
    });
    m.def("secp_seckey_valid", [](const py::bytes& key) {
        const std::string k = key;
        return k.size() == 32 && secp::seckey_valid(reinterpret_cast<const u8*>(k.data()));
    });
    // DER signature normalisation helpers used by policy and the GPU batch packer
    m.def("secp_der_to_rs", [](const py::bytes& sig) -> py::object {
        const std::string s = sig;
        secp::Scalar r, sv;
        if (!secp::sig_parse_der_lax(reinterpret_cast<const u8*>(s.data()), s.size(), r, sv)) return py::none();
        if (secp::sc_is_high(sv)) sv = secp::sc_neg(sv);
        u8 out[64];
        secp::sc_to_be(r, out);
        secp::sc_to_be(sv, out + 32);
        return pyb(out, 64);
    }, "lax-DER signature -> r || low-S s (32+32 bytes big-endian), None on a structural error");

    // ---------------------------------------------------------------- GPU batch verification
    m.attr("SECP_JOB_BYTES") = sizeof(SecpVerifyJob);
    m.def("secp_pack_jobs", [](const py::list& items) {
        // items: [(pubkey, der_sig_without_hashtype, msg32)] -> SecpVerifyJob array
        std::string out(items.size() * sizeof(SecpVerifyJob), '\0');
        auto* jobs = reinterpret_cast<SecpVerifyJob*>(&out[0]);
        size_t k = 0;
        for (auto it : items) {
            auto t = it.cast<py::tuple>();
            const std::string pub = t[0].cast<py::bytes>(), sig = t[1].cast<py::bytes>(),
                              msg = t[2].cast<py::bytes>();
            need32(msg, "msg");
            secp::pack_verify_job(reinterpret_cast<const u8*>(pub.data()), pub.size(),
                                  reinterpret_cast<const u8*>(sig.data()), sig.size(),
                                  reinterpret_cast<const u8*>(msg.data()), jobs[k++]);
        }
        return py::bytes(out);
    }, "pack (pubkey, DER signature, message) triples as gfx950 verify jobs");
    m.def("secp_gen_table32", [] {
        return py::bytes(reinterpret_cast<const char*>(secp::gen_table32()), 64 * 16 * 16 * 4);
    }, "the device comb table of G (64 KiB)");
    m.def("secp_verify_model32", [](const py::bytes& pub, const py::bytes& sig, const py::bytes& msg) {
        const std::string p = pub, sg = sig, m32 = msg;
        need32(m32, "msg");
        SecpVerifyJob job;
        secp::pack_verify_job(reinterpret_cast<const u8*>(p.data()), p.size(), reinterpret_cast<const u8*>(sg.data()),
                              sg.size(), reinterpret_cast<const u8*>(m32.data()), job);
        return secp::verify_job_model32(job);
    }, "the GPU verifier's 32-bit-limb arithmetic run on the host: 1 valid, 0 invalid, 2 degenerate");

    // ---------------------------------------------------------------- interpreter
    m.attr("SCRIPT_VERIFY_P2SH") = u32(SCRIPT_VERIFY_P2SH);
    m.attr("STANDARD_SCRIPT_VERIFY_FLAGS") = kStandardScriptFlags;
    m.attr("MANDATORY_SCRIPT_VERIFY_FLAGS") = kMandatoryScriptFlags;
    m.def("script_flag_bits", [] {
        py::dict d;
        const std::pair<const char*, u32> f[] = {
            {"NONE", SCRIPT_VERIFY_NONE}, {"P2SH", SCRIPT_VERIFY_P2SH}, {"STRICTENC", SCRIPT_VERIFY_STRICTENC},
            {"DERSIG", SCRIPT_VERIFY_DERSIG}, {"LOW_S", SCRIPT_VERIFY_LOW_S}, {"NULLDUMMY", SCRIPT_VERIFY_NULLDUMMY},
            {"SIGPUSHONLY", SCRIPT_VERIFY_SIGPUSHONLY}, {"MINIMALDATA", SCRIPT_VERIFY_MINIMALDATA},
            {"DISCOURAGE_UPGRADABLE_NOPS", SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_NOPS},
            {"CLEANSTACK", SCRIPT_VERIFY_CLEANSTACK}, {"CHECKLOCKTIMEVERIFY", SCRIPT_VERIFY_CHECKLOCKTIMEVERIFY},
            {"CHECKSEQUENCEVERIFY", SCRIPT_VERIFY_CHECKSEQUENCEVERIFY}, {"WITNESS", SCRIPT_VERIFY_WITNESS},
            {"DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM", SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM},
            {"MINIMALIF", SCRIPT_VERIFY_MINIMALIF}, {"NULLFAIL", SCRIPT_VERIFY_NULLFAIL},
            {"WITNESS_PUBKEYTYPE", SCRIPT_VERIFY_WITNESS_PUBKEYTYPE}};
        for (auto& [k, v] : f) d[k] = v;
        return d;
    }, "the reference's flag names (src/test/transaction_tests.cpp mapFlagNames)");
    m.def("verify_script", [](const py::bytes& script_sig, const py::bytes& script_pubkey,
                              const std::vector<py::bytes>& witness, u32 flags, const py::bytes& tx_raw, unsigned n_in,
                              int64_t amount, int sigcache) {
        const Transaction tx = tx_of(tx_raw);
        if (n_in >= tx.vin.size()) throw std::invalid_argument("input index out of range");
        const PrecomputedTx cache(tx);
        TxSigChecker checker(&tx, n_in, amount, &cache);
        if (sigcache < 0 || sigcache > 2) throw std::invalid_argument("sigcache: 0 none, 1 store, 2 use");
        checker.sigcache = TxSigChecker::CacheMode(sigcache);
        const std::vector<Bytes> wit = stack_of(witness);
        ScriptError err = ScriptError::UNKNOWN_ERROR;
        py::gil_scoped_release rel;
        const bool ok = verify_script(bytes_of(script_sig), bytes_of(script_pubkey), &wit, flags, checker, &err);
        py::gil_scoped_acquire acq;
        return py::make_tuple(ok, script_error_name(err));
    }, py::arg("script_sig"), py::arg("script_pubkey"), py::arg("witness"), py::arg("flags"), py::arg("tx"),
       py::arg("n_in"), py::arg("amount"), py::arg("sigcache") = 0,
       "VerifyScript of input n_in of the serialized tx -> (ok, error name); sigcache 1 = store verified "
       "signatures (mempool acceptance), 2 = answer from the cache (block validation)");
    m.def("sigcache_set_max_bytes", [](size_t b) { SigCache::instance().set_max_bytes(b); },
          "-maxsigcachesize (bytes of 32-byte entries)");
    m.def("sigcache_clear", [] { SigCache::instance().clear(); });
    m.def("sigcache_stats", [] {
        const SigCache::Stats s = SigCache::instance().stats();
        py::dict d;
        d["entries"] = s.entries;
        d["max_entries"] = s.max_entries;
        d["hits"] = s.hits;
        d["misses"] = s.misses;
        d["inserts"] = s.inserts;
        d["evictions"] = s.evictions;
        return d;
    });
    m.def("eval_script", [](const std::vector<py::bytes>& stack, const py::bytes& script, u32 flags) {
        std::vector<Bytes> st = stack_of(stack);
        ScriptError err = ScriptError::UNKNOWN_ERROR;
        const bool ok = eval_script(st, bytes_of(script), flags, SigChecker(), SigVersion::BASE, &err);
        py::list out;
        for (auto& e : st) out.append(pyb(e));
        return py::make_tuple(ok, script_error_name(err), out);
    }, "EvalScript with no transaction context (signature checks fail)");
    m.def("signature_hash", [](const py::bytes& script_code, const py::bytes& tx_raw, unsigned n_in, int hash_type,
                               int64_t amount, int sigversion) {
        const Transaction tx = tx_of(tx_raw);
        const Uint256 h = signature_hash(bytes_of(script_code), tx, n_in, hash_type, amount,
                                         sigversion ? SigVersion::WITNESS_V0 : SigVersion::BASE);
        return pyb(h.data, 32);
    }, py::arg("script_code"), py::arg("tx"), py::arg("n_in"), py::arg("hash_type"), py::arg("amount") = 0,
       py::arg("sigversion") = 0, "SignatureHash (uint256 storage order)");
    m.def("check_transaction", [](const py::bytes& tx_raw, const ChainParams* params, const assets::Flags* flags,
                                  bool block_check, bool mempool_check) {
        return check_transaction(tx_of(tx_raw), true, params ? &params->assets : nullptr, flags, block_check,
                                 mempool_check);
    }, py::arg("tx"), py::arg("params") = nullptr, py::arg("asset_flags") = nullptr, py::arg("block_check") = false,
       py::arg("mempool_check") = false, "CheckTransaction reject reason, '' when valid (asset rules with params)");
    m.def("script_sigop_count", [](const py::bytes& s, bool accurate) {
        return script_sigop_count(bytes_of(s), accurate);
    }, py::arg("script"), py::arg("accurate") = false);
    // ---------------------------------------------------------------- UTXO set / ConnectBlock
    m.attr("COINBASE_MATURITY") = kCoinbaseMaturity;
    m.attr("BLOCK_SCRIPT_VERIFY_FLAGS") = kBlockScriptFlags;
    py::class_<CoinsView, std::shared_ptr<CoinsView>>(m, "CoinsView")
        .def(py::init<>())
        .def("__len__", &CoinsView::size)
        .def("append_journal", &CoinsView::append_journal, py::call_guard<py::gil_scoped_release>(),
             "append the outputs added / spent since the last flush as one fsynced journal record")
        .def("load_with_journal", &CoinsView::load_with_journal, py::call_guard<py::gil_scoped_release>())
        .def("compact", &CoinsView::compact, py::call_guard<py::gil_scoped_release>(),
             "fold the journal into a fresh snapshot and truncate it")
        .def_property_readonly("dirty", &CoinsView::dirty)
        .def_readonly("journal_seq", &CoinsView::journal_seq)
        .def_readonly("replayed", &CoinsView::replayed)
        .def("get", [](const CoinsView& v, const py::bytes& txid, u32 n) -> py::object {
            OutPoint o;
            const std::string h = txid;
            need32(h, "txid");
            o.hash = Uint256::from_bytes(reinterpret_cast<const u8*>(h.data()));
            o.n = n;
            const Coin* c = v.find(o);
            if (!c) return py::none();
            return py::make_tuple(c->out.value, pyb(c->out.script_pubkey), c->height, c->coinbase);
        }, "(value, scriptPubKey, height, coinbase) of an unspent output, or None")
        .def("height_of_txid", [](const CoinsView& v, const py::bytes& txid) -> py::object {
            // AccessByTxid (src/coins.cpp): probe output indexes up to MAX_OUTPUTS_PER_BLOCK
            // (MAX_BLOCK_WEIGHT / (WITNESS_SCALE_FACTOR * size of an empty CTxOut))
            OutPoint o;
            const std::string h = txid;
            need32(h, "txid");
            o.hash = Uint256::from_bytes(reinterpret_cast<const u8*>(h.data()));
            for (o.n = 0; o.n < 8000000u / (4u * 9u); ++o.n)
                if (const Coin* c = v.find(o)) return py::int_(c->height);
            return py::none();
        }, "height of the block holding a transaction with an unspent output, or None")
        .def("add", [](CoinsView& v, const py::bytes& txid, u32 n, int64_t value, const py::bytes& spk, u32 height,
                       bool coinbase) {
            OutPoint o;
            const std::string h = txid;
            need32(h, "txid");
            o.hash = Uint256::from_bytes(reinterpret_cast<const u8*>(h.data()));
            o.n = n;
            Coin c;
            c.out.value = value;
            c.out.script_pubkey = bytes_of(spk);
            c.height = height;
            c.coinbase = coinbase;
            v.add(o, std::move(c));
        })
        .def_property("best_block", [](const CoinsView& v) { return pyb(v.best_block.data, 32); },
                      [](CoinsView& v, const py::bytes& b) {
                          const std::string h = b;
                          need32(h, "best_block");
                          v.best_block = Uint256::from_bytes(reinterpret_cast<const u8*>(h.data()));
                      })
        .def("spend", [](CoinsView& v, const py::bytes& txid, u32 n) {
            OutPoint o;
            const std::string h = txid;
            need32(h, "txid");
            o.hash = Uint256::from_bytes(reinterpret_cast<const u8*>(h.data()));
            o.n = n;
            return v.spend(o);
        }, "remove an unspent output (True if it existed)")
        .def("save", &CoinsView::save, py::call_guard<py::gil_scoped_release>())
        .def("load", &CoinsView::load, py::call_guard<py::gil_scoped_release>())
        .def("stats", [](const CoinsView& v) {
            const auto s = v.stats();
            return py::make_tuple(s.txouts, s.transactions, s.total, pyb(s.hash.data, 32), s.bogosize);
        }, "(txouts, transactions, total amount, hash_serialized_2, bogosize)")
        .def("outputs_for_scripts", [](const CoinsView& v, const std::vector<py::bytes>& spks) {
            std::set<Bytes> want;
            for (auto& s : spks) want.insert(bytes_of(s));
            py::list out;
            v.for_each([&](const OutPoint& o, const Coin& c) {
                if (want.count(c.out.script_pubkey))
                    out.append(py::make_tuple(pyb(o.hash.data, 32), o.n, c.out.value, pyb(c.out.script_pubkey),
                                              c.height, c.coinbase));
            });
            return out;
        }, "unspent outputs paying any of these scriptPubKeys: (txid, n, value, spk, height, coinbase)")
        .def("asset_outputs", [](const CoinsView& v, py::object hashes) {
            // asset scripts (P2PKH prefix + OP_CLORE_ASSET payload) of these hash160s, or of all when None
            std::set<std::string> want;
            const bool all = hashes.is_none();
            if (!all)
                for (auto& h : hashes.cast<std::vector<py::bytes>>()) want.insert(std::string(h));
            py::list out;
            v.for_each([&](const OutPoint& o, const Coin& c) {
                const Bytes& s = c.out.script_pubkey;
                if (assets::asset_script_kind(s) == assets::OutKind::NONE) return;
                if (!all && !want.count(std::string(reinterpret_cast<const char*>(s.data() + 3), 20))) return;
                out.append(py::make_tuple(pyb(o.hash.data, 32), o.n, c.out.value, pyb(s), c.height, c.coinbase));
            });
            return out;
        }, py::arg("hashes") = py::none(),
           "unspent asset outputs to these hash160s (all when None): (txid, n, value, spk, height, coinbase)");
    py::class_<ConnectResult>(m, "ConnectResult")
        .def_readonly("ok", &ConnectResult::ok)
        .def_readonly("reject", &ConnectResult::reject)
        .def_readonly("dos", &ConnectResult::dos)
        .def_readonly("fees", &ConnectResult::fees)
        .def_readonly("sigop_cost", &ConnectResult::sigop_cost)
        .def_readonly("sig_at", &ConnectResult::sig_at)
        .def_property_readonly("asset_undo", [](const ConnectResult& r) { return pyb(r.asset_undo); })
        .def_property_readonly("num_sigs", [](const ConnectResult& r) { return r.sigs.size(); })
        .def("sig_items", [](const ConnectResult& r) {
            py::list out;
            for (auto& p : r.sigs) out.append(py::make_tuple(pyb(p.pubkey), pyb(p.sig), pyb(p.msg.data, 32)));
            return out;
        }, "deferred signatures as (pubkey, DER signature, message) for ops/secp.verify_batch");
    m.def("connect_block", [](const Block& block, int height, CoinsView& view, bool check_scripts, bool defer_sigs,
                              py::object mtp_at, int64_t block_mtp, u32 flags, int threads, assets::State* asset_state,
                              const assets::Flags& asset_flags, const py::bytes& block_hash, bool sigcache) {
        ConnectOptions opt;
        opt.assets = asset_state;
        opt.asset_flags = asset_flags;
        const std::string bh = block_hash;
        if (bh.size() == 32) opt.block_hash = Uint256::from_bytes(reinterpret_cast<const u8*>(bh.data()));
        opt.script_flags = flags;
        opt.check_scripts = check_scripts;
        opt.defer_sigs = defer_sigs;
        opt.sigcache = sigcache;
        opt.block_mtp = block_mtp;
        opt.threads = threads;
        if (!mtp_at.is_none())
            opt.mtp_at = [mtp_at](int h) {
                py::gil_scoped_acquire gil;
                return mtp_at(h).cast<int64_t>();
            };
        BlockUndo undo;
        ConnectResult r;
        Bytes ub;
        {
            py::gil_scoped_release rel;  // the UTXO pass and the script-check threads run without the GIL
            r = connect_block(block, height, view, opt, undo);
            if (r.ok) ub = serialize_block_undo(undo);
        }
        return py::make_tuple(std::move(r), pyb(ub));
    }, py::arg("block"), py::arg("height"), py::arg("view"), py::arg("check_scripts") = true,
       py::arg("defer_sigs") = false, py::arg("mtp_at") = py::none(), py::arg("block_mtp") = 0,
       py::arg("flags") = kBlockScriptFlags, py::arg("threads") = 1, py::arg("assets") = nullptr,
       py::arg("asset_flags") = assets::Flags{}, py::arg("block_hash") = py::bytes(), py::arg("sigcache") = true,
       "ConnectBlock against the view -> (ConnectResult, serialized CBlockUndo); the view is unchanged on failure");
    m.def("disconnect_block", [](const Block& block, const py::bytes& undo, CoinsView& view, assets::State* st,
                                 const py::bytes& asset_undo) {
        const Bytes au = bytes_of(asset_undo);
        return disconnect_block(block, deserialize_block_undo(bytes_of(undo)), view, st, &au);
    }, py::arg("block"), py::arg("undo"), py::arg("view"), py::arg("assets") = nullptr, py::arg("asset_undo") = py::bytes(),
       "DisconnectBlock with its undo data: False if they did not match the view (it is still reverted)");
    py::class_<ChainIndexes, std::shared_ptr<ChainIndexes>>(m, "ChainIndexes")
        .def(py::init([](bool tx, bool addr, bool spent, bool ts) {
                 auto x = std::make_shared<ChainIndexes>();
                 x->txindex = tx;
                 x->addressindex = addr;
                 x->spentindex = spent;
                 x->timestampindex = ts;
                 return x;
             }),
             py::arg("txindex") = false, py::arg("addressindex") = false, py::arg("spentindex") = false,
             py::arg("timestampindex") = false)
        .def_readonly("txindex", &ChainIndexes::txindex)
        .def_readonly("addressindex", &ChainIndexes::addressindex)
        .def_readonly("spentindex", &ChainIndexes::spentindex)
        .def_readonly("timestampindex", &ChainIndexes::timestampindex)
        .def_property("best_block", [](const ChainIndexes& x) { return pyb(x.best_block.data, 32); },
                      [](ChainIndexes& x, const py::bytes& b) {
                          const std::string h = b;
                          need32(h, "best_block");
                          x.best_block = Uint256::from_bytes(reinterpret_cast<const u8*>(h.data()));
                      })
        .def("connect", [](ChainIndexes& x, const Block& b, int height, const py::bytes& hash, const py::bytes& undo,
                           int file, u32 data_pos) {
            const std::string h = hash;
            need32(h, "hash");
            x.connect(b, height, Uint256::from_bytes(reinterpret_cast<const u8*>(h.data())),
                      deserialize_block_undo(bytes_of(undo)), file, data_pos);
        }, py::arg("block"), py::arg("height"), py::arg("hash"), py::arg("undo"), py::arg("file") = -1,
           py::arg("data_pos") = 0)
        .def_readwrite("journal", &ChainIndexes::journal)
        .def_property_readonly("pending_changes", &ChainIndexes::pending_changes)
        .def("disconnect", [](ChainIndexes& x, const Block& b, int height, const py::bytes& hash, const py::bytes& undo) {
            const std::string h = hash;
            need32(h, "hash");
            x.disconnect(b, height, Uint256::from_bytes(reinterpret_cast<const u8*>(h.data())),
                         deserialize_block_undo(bytes_of(undo)));
        })
        .def("tx_block", [](const ChainIndexes& x, const py::bytes& txid) -> py::object {
            const std::string t = txid;
            need32(t, "txid");
            const Uint256* b = x.tx_block(Uint256::from_bytes(reinterpret_cast<const u8*>(t.data())));
            if (!b) return py::none();
            return pyb(b->data, 32);
        })
        .def("deltas", [](const ChainIndexes& x, int type, const py::bytes& h160, const std::string& asset, int start,
                          int end) {
            const std::string h = h160;
            if (h.size() != 20) throw std::invalid_argument("hash160 must be 20 bytes");
            py::list out;
            for (auto& [name, d] : x.deltas(type, reinterpret_cast<const u8*>(h.data()), asset, start, end))
                out.append(py::make_tuple(name, d.height, d.tx_index, pyb(d.txid.data, 32), d.index, d.spending, d.amount));
            return out;
        }, py::arg("type"), py::arg("hash160"), py::arg("asset") = "CLORE", py::arg("start") = 0, py::arg("end") = 0,
           "[(asset, height, tx index, txid, index, spending, amount)] in chain order")
        .def("unspent", [](const ChainIndexes& x, int type, const py::bytes& h160, const std::string& asset) {
            const std::string h = h160;
            if (h.size() != 20) throw std::invalid_argument("hash160 must be 20 bytes");
            py::list out;
            for (auto& [name, u] : x.unspent(type, reinterpret_cast<const u8*>(h.data()), asset))
                out.append(py::make_tuple(name, pyb(u.txid.data, 32), u.index, u.amount, pyb(u.script), u.height));
            return out;
        }, py::arg("type"), py::arg("hash160"), py::arg("asset") = "CLORE",
           "[(asset, txid, index, amount, script, height)] by height")
        .def("spent", [](const ChainIndexes& x, const py::bytes& txid, u32 n) -> py::object {
            const std::string t = txid;
            need32(t, "txid");
            const SpentInfo* s = x.spent(Uint256::from_bytes(reinterpret_cast<const u8*>(t.data())), n);
            if (!s) return py::none();
            return py::make_tuple(pyb(s->txid.data, 32), s->input, s->height, s->amount, s->addr_type, pyb(s->h160, 20));
        })
        .def("timestamps", [](const ChainIndexes& x, u32 low, u32 high) {
            py::list out;
            for (auto& h : x.timestamps(low, high)) out.append(pyb(h.data, 32));
            return out;
        })
        .def("serialize", [](const ChainIndexes& x) { return pyb(x.serialize()); })
        .def("deserialize", [](ChainIndexes& x, const py::bytes& b) { return x.deserialize(bytes_of(b)); });
    m.def("verify_input_host", [](const Block& block, u32 tx_index, u32 n_in, int64_t value, const py::bytes& spk,
                                  u32 flags) {
        if (tx_index >= block.vtx.size() || n_in >= block.vtx[tx_index].vin.size())
            throw std::invalid_argument("no such input");
        Coin c;
        c.out.value = value;
        c.out.script_pubkey = bytes_of(spk);
        ScriptError err = ScriptError::UNKNOWN_ERROR;
        const bool ok = verify_input_host(block.vtx[tx_index], n_in, c, flags, &err);
        return py::make_tuple(ok, script_error_name(err));
    });
    m.def("block_undo_coin", [](const py::bytes& undo, u32 tx_index, u32 n_in) {
        const BlockUndo u = deserialize_block_undo(bytes_of(undo));
        if (tx_index == 0 || tx_index > u.vtxundo.size() || n_in >= u.vtxundo[tx_index - 1].prev.size())
            throw std::invalid_argument("no such spent coin in the undo data");
        const Coin& c = u.vtxundo[tx_index - 1].prev[n_in];
        return py::make_tuple(c.out.value, pyb(c.out.script_pubkey), c.height, c.coinbase);
    }, "the coin input n_in of transaction tx_index spent, from a block's undo data");
    m.def("block_undo_roundtrip", [](const py::bytes& b) {
        return pyb(serialize_block_undo(deserialize_block_undo(bytes_of(b))));
    });
    m.def("compress_amount", &compress_amount);
    m.def("decompress_amount", &decompress_amount);
    m.def("tx_legacy_sigops", [](const py::bytes& tx_raw) { return tx_legacy_sigops(tx_of(tx_raw)); },
          "GetLegacySigOpCount of a transaction (no spent outputs needed)");
    m.def("tx_sigop_cost", [](const py::bytes& tx_raw, const std::vector<py::bytes>& spent_spks, u32 flags) {
        const Transaction tx = tx_of(tx_raw);
        std::vector<Coin> coins(spent_spks.size());
        std::vector<const Coin*> ptrs;
        for (size_t i = 0; i < spent_spks.size(); ++i) {
            coins[i].out.script_pubkey = bytes_of(spent_spks[i]);
            ptrs.push_back(&coins[i]);
        }
        return tx_sigop_cost(tx, ptrs, flags);
    }, "GetTransactionSigOpCost: legacy x4 + P2SH redeem x4 + witness, given the spent scriptPubKeys");

    m.def("script_is_push_only", [](const py::bytes& s) { return script_is_push_only(bytes_of(s)); });
    m.def("is_valid_signature_encoding", [](const py::bytes& s) { return is_valid_signature_encoding(bytes_of(s)); });
}
