// pybind11 module `_core`: the CPU consensus/PoW core exposed to Python.
// All 32/64-byte hashes cross the boundary as `bytes` in storage order.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../crypto/keccak.hpp"
#include "../crypto/sha256.hpp"
#include "../pow/ethash.hpp"
#include "../pow/kawpow.hpp"

namespace py = pybind11;
using namespace nodexa;

namespace {

Hash256 to_h256(const py::bytes& b) {
    std::string s = b;
    if (s.size() != 32) throw std::invalid_argument("expected 32 bytes");
    Hash256 h;
    std::memcpy(h.bytes, s.data(), 32);
    return h;
}
py::bytes from_h256(const Hash256& h) { return py::bytes(reinterpret_cast<const char*>(h.bytes), 32); }
py::bytes from_h512(const Hash512& h) { return py::bytes(reinterpret_cast<const char*>(h.bytes), 64); }
std::string as_str(const py::bytes& b) { return std::string(b); }

}  // namespace

void bind_extra(py::module_& m);  // bind_extra.cpp: chain, X16R, Equihash
void bind_script(py::module_& m);  // bind_script.cpp: secp256k1, script interpreter
void bind_assets(py::module_& m);  // bind_assets.cpp: asset layer
void bind_fees(py::module_& m);    // bind_fees.cpp: fee estimator
void bind_store(py::module_& m);   // bind_store.cpp: LevelDB-format store

PYBIND11_MODULE(_core, m) {
    m.doc() = "nodexa native CPU core: crypto, ethash/KawPow golden model, Equihash, consensus";

    // ---------------- crypto ----------------
    m.def("keccak256", [](const py::bytes& d) { auto s = as_str(d); return from_h256(keccak256((const u8*)s.data(), s.size())); });
    m.def("keccak512", [](const py::bytes& d) { auto s = as_str(d); return from_h512(keccak512((const u8*)s.data(), s.size())); });
    m.def("keccakf800", [](std::vector<u32> st) {
        if (st.size() != 25) throw std::invalid_argument("state must have 25 words");
        keccakf800(st.data());
        return st;
    });
    m.def("keccakf1600", [](std::vector<u64> st) {
        if (st.size() != 25) throw std::invalid_argument("state must have 25 words");
        keccakf1600(st.data());
        return st;
    });
    m.def("sha256", [](const py::bytes& d) { auto s = as_str(d); u8 o[32]; sha256((const u8*)s.data(), s.size(), o); return py::bytes((char*)o, 32); });
    m.def("sha256d", [](const py::bytes& d) { auto s = as_str(d); u8 o[32]; sha256d((const u8*)s.data(), s.size(), o); return py::bytes((char*)o, 32); });
    m.def("hash_le", [](const py::bytes& a, const py::bytes& b) { return hash_le(to_h256(a), to_h256(b)); },
          "big-endian a <= b over 32-byte hashes (ethash is_less_or_equal)");

    // ---------------- ethash ----------------
    m.attr("EPOCH_LENGTH") = kEpochLength;
    m.def("find_largest_prime", &find_largest_prime);
    m.def("light_cache_num_items", &light_cache_num_items);
    m.def("full_dataset_num_items", &full_dataset_num_items);
    m.def("epoch_seed", [](int e) { return from_h256(epoch_seed(e)); });
    m.def("find_epoch_number", [](const py::bytes& s) { return find_epoch_number(to_h256(s)); });

    py::class_<EpochContext, std::shared_ptr<EpochContext>>(m, "EpochContext")
        .def_readonly("epoch", &EpochContext::epoch)
        .def_readonly("light_items", &EpochContext::light_items)
        .def_readonly("full_items", &EpochContext::full_items)
        .def_property_readonly("light_bytes", &EpochContext::light_bytes)
        .def_property_readonly("full_bytes", &EpochContext::full_bytes)
        .def_property_readonly("l1", [](const EpochContext& c) { return std::vector<u32>(c.l1.begin(), c.l1.end()); })
        .def("light_cache", [](const EpochContext& c) {
            return py::bytes(reinterpret_cast<const char*>(c.light.data()), c.light.size() * 64);
        }, "raw light cache (light_items x 64 bytes)")
        .def("light_cache_ptr", [](const EpochContext& c) { return reinterpret_cast<uintptr_t>(c.light.data()); });
    m.def("set_light_cache_dir", &set_light_cache_dir, "-dagcache: on-disk light-cache cache directory ('' = off)");
    m.def("light_cache_dir", &light_cache_dir);
    m.def("create_epoch_context", [](int e) { return std::const_pointer_cast<EpochContext>(create_epoch_context(e)); },
          py::call_guard<py::gil_scoped_release>(), "uncached build (tests); honours the on-disk cache");
    m.def("get_epoch_context", [](int e) { return std::const_pointer_cast<EpochContext>(get_epoch_context(e)); },
          py::call_guard<py::gil_scoped_release>());
    m.def("dataset_item_512", [](const EpochContext& c, u64 i) { return from_h512(dataset_item_512(c, i)); });
    m.def("dataset_item_2048", [](const EpochContext& c, u32 i) {
        Hash512 it[4];
        dataset_item_2048(c, i, it);
        return py::bytes(reinterpret_cast<const char*>(it), 256);
    });
    m.def("ethash_hash", [](const EpochContext& c, const py::bytes& h, u64 n) {
        auto r = ethash_hash(c, to_h256(h), n);
        return py::make_tuple(from_h256(r.final_hash), from_h256(r.mix_hash));
    });
    m.def("ethash_verify", [](const EpochContext& c, const py::bytes& h, const py::bytes& mix, u64 n, const py::bytes& b) {
        return ethash_verify(c, to_h256(h), to_h256(mix), n, to_h256(b));
    });

    py::class_<HostDag, std::shared_ptr<HostDag>>(m, "HostDag")
        .def(py::init([](std::shared_ptr<EpochContext> c) { return std::make_shared<HostDag>(c); }))
        .def("build_all", &HostDag::build_all, py::call_guard<py::gil_scoped_release>())
        .def_property_readonly("num_items512", &HostDag::num_items512);

    // ---------------- KawPow ----------------
    py::class_<KawpowProgram>(m, "KawpowProgram")
        .def_readonly("period", &KawpowProgram::period)
        .def("cache_ops", [](const KawpowProgram& p) {
            py::list l;
            for (auto& c : p.cache) l.append(py::make_tuple(c.src, c.dst, c.sel));
            return l;
        })
        .def("math_ops", [](const KawpowProgram& p) {
            py::list l;
            for (auto& o : p.math) l.append(py::make_tuple(o.src1, o.src2, o.sel1, o.dst, o.sel2));
            return l;
        })
        .def("dag_ops", [](const KawpowProgram& p) {
            py::list l;
            for (int i = 0; i < kDagLoads; ++i) l.append(py::make_tuple(p.dag_dst[i], p.dag_sel[i]));
            return l;
        });
    m.def("make_kawpow_program", &make_kawpow_program);
    m.def("kawpow_codegen_hip", [](u64 period) { return kawpow_codegen_hip(make_kawpow_program(period)); });
    m.def("kawpow_program_words", [](u64 period) { return kawpow_program_words(make_kawpow_program(period)); });
    m.def("kawpow_hash", [](const EpochContext& c, int block, const py::bytes& h, u64 nonce) {
        KawpowResult r;
        Hash256 hh = to_h256(h);
        {
            py::gil_scoped_release rel;
            r = kawpow_hash(c, block, hh, nonce);
        }
        return py::make_tuple(from_h256(r.final_hash), from_h256(r.mix_hash));
    });
    m.def("kawpow_hash_full", [](HostDag& d, int block, const py::bytes& h, u64 nonce) {
        auto r = kawpow_hash_full(d, block, to_h256(h), nonce);
        return py::make_tuple(from_h256(r.final_hash), from_h256(r.mix_hash));
    });
    m.def("kawpow_verify", [](const EpochContext& c, int block, const py::bytes& h, const py::bytes& mix, u64 nonce,
                              const py::bytes& boundary) {
        Hash256 hh = to_h256(h), mm = to_h256(mix), bb = to_h256(boundary);
        py::gil_scoped_release rel;
        return kawpow_verify(c, block, hh, mm, nonce, bb);
    });
    m.def("kawpow_hash_no_verify", [](int block, const py::bytes& h, const py::bytes& mix, u64 nonce) {
        return from_h256(kawpow_hash_no_verify(block, to_h256(h), to_h256(mix), nonce));
    });
    m.def("kawpow_initial_state", [](const py::bytes& h, u64 nonce) {
        std::vector<u32> s(8);
        kawpow_initial_state(to_h256(h), nonce, s.data());
        return s;
    });
    auto search_tuple = [](const KawpowSearchResult& r) {
        return py::make_tuple(r.found, r.nonce, from_h256(r.result.final_hash), from_h256(r.result.mix_hash));
    };
    m.def("kawpow_search_light", [search_tuple](const EpochContext& c, int block, const py::bytes& h, const py::bytes& b,
                                                u64 start, u64 iters) {
        Hash256 hh = to_h256(h), bb = to_h256(b);
        KawpowSearchResult r;
        {
            py::gil_scoped_release rel;
            r = kawpow_search_light(c, block, hh, bb, start, iters);
        }
        return search_tuple(r);
    });
    m.def("kawpow_search_full", [search_tuple](HostDag& d, int block, const py::bytes& h, const py::bytes& b, u64 start,
                                               u64 iters, int threads) {
        Hash256 hh = to_h256(h), bb = to_h256(b);
        KawpowSearchResult r;
        {
            py::gil_scoped_release rel;
            r = kawpow_search_full(d, block, hh, bb, start, iters, threads);
        }
        return search_tuple(r);
    });
    m.def("kawpow_cpu_hashrate", &kawpow_cpu_hashrate, py::call_guard<py::gil_scoped_release>());

    bind_assets(m);  // first: AssetFlags is a default argument of later bindings
    bind_extra(m);
    bind_script(m);
    bind_fees(m);
    bind_store(m);
}
