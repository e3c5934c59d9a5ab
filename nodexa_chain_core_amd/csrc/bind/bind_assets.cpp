// Bindings for the asset layer (chain/assets.*): names, scripts, the asset state and the
// consensus checks. Asset addresses cross the boundary as 20-byte hash160 values.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../chain/assets.hpp"
#include "../chain/coins.hpp"
#include "../chain/params.hpp"

namespace py = pybind11;
using namespace nodexa;

namespace {

Bytes bytes_of(const py::bytes& b) {
    std::string s = b;
    return Bytes(s.begin(), s.end());
}
py::bytes pyb(const std::string& s) { return py::bytes(s); }
py::bytes pyb(const Bytes& b) { return py::bytes(reinterpret_cast<const char*>(b.data()), b.size()); }

void h160_of(const py::bytes& b, u8 out[20]) {
    const std::string s = b;
    if (s.size() != 20) throw std::invalid_argument("hash160 must be 20 bytes");
    std::memcpy(out, s.data(), 20);
}

Transaction tx_of(const py::bytes& raw) {
    const Bytes b = bytes_of(raw);
    Reader r(b);
    Transaction tx = Transaction::deserialize(r, true);
    if (!r.empty()) throw std::invalid_argument("trailing bytes after transaction");
    return tx;
}

const char* out_kind_name(assets::OutKind k) {
    switch (k) {
        case assets::OutKind::NEW: return "new_asset";
        case assets::OutKind::OWNER: return "owner";
        case assets::OutKind::TRANSFER: return "transfer_asset";
        case assets::OutKind::REISSUE: return "reissue_asset";
        default: return "";
    }
}

py::dict meta_dict(const assets::Meta& m) {
    py::dict d;
    d["name"] = m.name;
    d["amount"] = m.amount;
    d["units"] = m.units;
    d["reissuable"] = m.reissuable;
    d["has_ipfs"] = m.has_ipfs;
    d["ipfs"] = pyb(m.ipfs);
    d["height"] = m.height;
    d["block"] = py::bytes(reinterpret_cast<const char*>(m.block.data), 32);
    return d;
}

}  // namespace

void bind_assets(py::module_& m) {
    py::class_<assets::Flags>(m, "AssetFlags")
        .def(py::init([](bool a, bool mr, bool ev, bool cb) {
                 assets::Flags f;
                 f.assets = a;
                 f.msg_restricted = mr;
                 f.enforce_values = ev;
                 f.coinbase_assets = cb;
                 return f;
             }),
             py::arg("assets") = false, py::arg("msg_restricted") = false, py::arg("enforce_values") = false,
             py::arg("coinbase_assets") = false)
        .def_readwrite("assets", &assets::Flags::assets)
        .def_readwrite("msg_restricted", &assets::Flags::msg_restricted)
        .def_readwrite("enforce_values", &assets::Flags::enforce_values)
        .def_readwrite("coinbase_assets", &assets::Flags::coinbase_assets);

    m.def("asset_name_type", [](const std::string& name) {
        std::string err;
        const assets::Type t = assets::name_type(name, &err);
        return py::make_tuple(std::string(assets::type_name(t)), err);
    }, "IsAssetNameValid -> (type name or 'INVALID', error)");
    m.def("asset_parent_name", &assets::parent_name);
    m.def("asset_amount_fits_units", &assets::amount_fits_units);
    m.def("bool_expr", [](const std::string& e, const std::map<std::string, bool>& vals) {
        return assets::bool_expr(e, vals);
    }, "LibBoolEE::resolve (raises RuntimeError on a syntax error or an unknown variable)");
    m.def("check_verifier_string", [](const std::string& v) {
        std::set<std::string> found;
        std::string err;
        const bool ok = assets::check_verifier(v, found, err);
        return py::make_tuple(ok, err, found);
    });
    m.def("strip_verifier_string", &assets::strip_verifier);
    m.def("encode_asset_data", [](const py::bytes& raw) { return assets::encode_asset_data(std::string(raw)); });
    m.def("decode_asset_data", [](const std::string& s) { return pyb(assets::decode_asset_data(s)); });

    m.def("parse_asset_script", [](const py::bytes& spk) -> py::object {
        assets::AssetOut a;
        if (!assets::parse_asset_out(bytes_of(spk), a)) return py::none();
        py::dict d;
        d["type"] = out_kind_name(a.kind);
        d["hash160"] = py::bytes(reinterpret_cast<const char*>(a.h160), 20);
        d["name"] = a.name;
        d["amount"] = a.amount;
        d["units"] = a.units;
        d["reissuable"] = a.reissuable;
        d["has_ipfs"] = a.has_ipfs;
        d["ipfs"] = pyb(a.ipfs);
        d["message"] = pyb(a.message);
        d["expire"] = a.expire;
        return d;
    }, "the decoded asset payload of a scriptPubKey, or None");
    m.def("parse_null_asset_script", [](const py::bytes& spk) -> py::object {
        const Bytes s = bytes_of(spk);
        py::dict d;
        std::string name, v;
        int flag = 0;
        u8 h[20];
        switch (assets::null_kind(s)) {
            case assets::NullKind::TAG:
                if (!assets::parse_null_tag(s, name, flag, h)) return py::none();
                d["type"] = "tag";
                d["hash160"] = py::bytes(reinterpret_cast<const char*>(h), 20);
                d["name"] = name;
                d["flag"] = flag;
                return d;
            case assets::NullKind::GLOBAL:
                if (!assets::parse_null_global(s, name, flag)) return py::none();
                d["type"] = "global";
                d["name"] = name;
                d["flag"] = flag;
                return d;
            case assets::NullKind::VERIFIER:
                if (!assets::parse_null_verifier(s, v)) return py::none();
                d["type"] = "verifier";
                d["verifier"] = v;
                return d;
            default: return py::none();
        }
    });
    m.def("script_unspendable", [](const py::bytes& spk) { return assets::script_unspendable(bytes_of(spk)); });

    m.def("asset_script_new", [](const py::bytes& h, const std::string& name, int64_t amount, int units, int reissuable,
                                 const py::bytes& ipfs) {
        u8 hb[20];
        h160_of(h, hb);
        assets::AssetOut a;
        a.name = name;
        a.amount = amount;
        a.units = units;
        a.reissuable = reissuable;
        a.ipfs = std::string(ipfs);
        a.has_ipfs = a.ipfs.empty() ? 0 : 1;
        return pyb(assets::script_new(hb, a));
    }, py::arg("hash160"), py::arg("name"), py::arg("amount"), py::arg("units") = 0, py::arg("reissuable") = 1,
       py::arg("ipfs") = py::bytes());
    m.def("asset_script_owner", [](const py::bytes& h, const std::string& name) {
        u8 hb[20];
        h160_of(h, hb);
        return pyb(assets::script_owner(hb, name));
    });
    m.def("asset_script_transfer", [](const py::bytes& h, const std::string& name, int64_t amount,
                                      const py::bytes& message, int64_t expire) {
        u8 hb[20];
        h160_of(h, hb);
        return pyb(assets::script_transfer(hb, name, amount, std::string(message), expire));
    }, py::arg("hash160"), py::arg("name"), py::arg("amount"), py::arg("message") = py::bytes(), py::arg("expire") = 0);
    m.def("asset_script_reissue", [](const py::bytes& h, const std::string& name, int64_t amount, int units,
                                     int reissuable, const py::bytes& ipfs) {
        u8 hb[20];
        h160_of(h, hb);
        return pyb(assets::script_reissue(hb, name, amount, units, reissuable, std::string(ipfs)));
    }, py::arg("hash160"), py::arg("name"), py::arg("amount"), py::arg("units") = -1, py::arg("reissuable") = 1,
       py::arg("ipfs") = py::bytes());
    m.def("asset_script_null_tag", [](const py::bytes& h, const std::string& name, int flag) {
        u8 hb[20];
        h160_of(h, hb);
        return pyb(assets::script_null_tag(hb, name, flag));
    });
    m.def("asset_script_null_global", [](const std::string& name, int flag) {
        return pyb(assets::script_null_global(name, flag));
    });
    m.def("asset_script_null_verifier", [](const std::string& v) { return pyb(assets::script_null_verifier(v)); });

    m.def("asset_tx_kind", [](const py::bytes& raw) {
        static const char* names[] = {"", "new", "new_unique", "new_msgchannel", "new_qualifier", "new_restricted",
                                      "reissue"};
        return std::string(names[int(assets::tx_kind(tx_of(raw)))]);
    });
    m.def("check_tx_assets", [](const py::bytes& raw, const std::vector<py::tuple>& spent, const assets::State& st,
                                const assets::Flags& f, const std::set<std::string>& pending) {
        // spent: (value, scriptPubKey) of every input, in input order
        std::vector<Coin> coins(spent.size());
        std::vector<const Coin*> ptrs;
        for (size_t i = 0; i < spent.size(); ++i) {
            coins[i].out.value = spent[i][0].cast<int64_t>();
            coins[i].out.script_pubkey = bytes_of(spent[i][1].cast<py::bytes>());
            ptrs.push_back(&coins[i]);
        }
        return assets::check_tx_contextual(tx_of(raw), ptrs, st, f, &pending);
    }, py::arg("tx"), py::arg("spent"), py::arg("state"), py::arg("flags"), py::arg("pending_names") = std::set<std::string>{},
       "Consensus::CheckTxAssets (mempool form): '' or the reject reason");

    py::class_<assets::State, std::shared_ptr<assets::State>>(m, "AssetsState")
        .def(py::init<>())
        .def("get", [](const assets::State& s, const std::string& name) -> py::object {
            const assets::Meta* meta = s.find(name);
            if (!meta) return py::none();
            return meta_dict(*meta);
        })
        .def("__len__", [](const assets::State& s) { return s.metas().size(); })
        .def("mark_all_dirty", &assets::State::mark_all_dirty)
        .def("dirty_count", &assets::State::dirty_count)
        .def("names", [](const assets::State& s) {
            std::vector<std::string> out;
            for (auto& kv : s.metas()) out.push_back(kv.first);
            return out;
        })
        .def("balance", [](const assets::State& s, const std::string& name, const py::bytes& h) {
            u8 hb[20];
            h160_of(h, hb);
            return s.balance(name, hb);
        })
        .def("balances", [](const assets::State& s) {
            py::list out;
            for (auto& [k, v] : s.balances()) out.append(py::make_tuple(k.first, pyb(k.second), v));
            return out;
        }, "[(asset, hash160, amount)]")
        .def("tags", [](const assets::State& s) {
            py::list out;
            for (auto& k : s.tags()) out.append(py::make_tuple(k.first, pyb(k.second)));
            return out;
        })
        .def("restrictions", [](const assets::State& s) {
            py::list out;
            for (auto& k : s.restrictions()) out.append(py::make_tuple(k.first, pyb(k.second)));
            return out;
        })
        .def("global_restrictions", [](const assets::State& s) {
            return std::vector<std::string>(s.global_restrictions().begin(), s.global_restrictions().end());
        })
        .def("verifier", [](const assets::State& s, const std::string& name) -> py::object {
            const std::string* v = s.verifier(name);
            if (!v) return py::none();
            return py::str(*v);
        })
        .def("has_tag", [](const assets::State& s, const std::string& q, const py::bytes& h) {
            u8 hb[20];
            h160_of(h, hb);
            return s.has_tag(q, hb);
        })
        .def("is_frozen", [](const assets::State& s, const std::string& r, const py::bytes& h) {
            u8 hb[20];
            h160_of(h, hb);
            return s.frozen(r, hb);
        })
        .def("is_global_frozen", &assets::State::global_frozen)
        .def("undo", [](assets::State& s, const py::bytes& rec) { return s.undo(bytes_of(rec)); })
        .def_property("best_block",
                      [](const assets::State& s) { return py::bytes(reinterpret_cast<const char*>(s.best_block.data), 32); },
                      [](assets::State& s, const py::bytes& b) {
                          const std::string h = b;
                          if (h.size() != 32) throw std::invalid_argument("best_block must be 32 bytes");
                          s.best_block = Uint256::from_bytes(reinterpret_cast<const u8*>(h.data()));
                      })
        .def("serialize", [](const assets::State& s) { return pyb(s.serialize()); })
        .def("deserialize", [](assets::State& s, const py::bytes& b) { return s.deserialize(bytes_of(b)); });

    m.def("asset_burn_info", [](const ChainParams& p) {
        py::dict d;
        const char* keys[10] = {"root", "reissue", "sub", "unique", "msgchannel", "qualifier", "subqualifier",
                                "restricted", "tag", "global"};
        const assets::Params& a = p.assets;
        const int64_t amounts[10] = {a.burn_root, a.burn_reissue, a.burn_sub, a.burn_unique, a.burn_msgchannel,
                                     a.burn_qualifier, a.burn_subqualifier, a.burn_restricted, a.burn_tag, 0};
        for (int i = 0; i < 10; ++i) d[keys[i]] = py::make_tuple(p.asset_burn_addresses[i], amounts[i]);
        return d;
    }, "{kind: (burn address, burn amount)}");
}
