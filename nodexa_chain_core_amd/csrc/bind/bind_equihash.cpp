// Bindings for the Equihash CPU golden model and BLAKE2b.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../crypto/blake2b.hpp"
#include "../pow/equihash.hpp"

namespace py = pybind11;
using namespace nodexa;

void bind_equihash_cpu(py::module_& m) {
    m.def("blake2b", [](const py::bytes& d, size_t outlen, const py::object& personal) {
        std::string s = d;
        std::string pers;
        if (!personal.is_none()) {
            pers = personal.cast<std::string>();
            if (pers.size() != 16) throw std::invalid_argument("personal must be 16 bytes");
        }
        Blake2b st(outlen, pers.empty() ? nullptr : reinterpret_cast<const u8*>(pers.data()));
        st.update(reinterpret_cast<const u8*>(s.data()), s.size());
        u8 out[64];
        st.final(out);
        return py::bytes(reinterpret_cast<const char*>(out), outlen);
    }, py::arg("data"), py::arg("outlen") = 64, py::arg("personal") = py::none());

    py::class_<EquihashParams>(m, "EquihashParams")
        .def(py::init([](int n, int k) { EquihashParams p; p.n = n; p.k = k; return p; }), py::arg("n") = 200, py::arg("k") = 9)
        .def_readonly("n", &EquihashParams::n)
        .def_readonly("k", &EquihashParams::k)
        .def_property_readonly("collision_bits", &EquihashParams::collision_bits)
        .def_property_readonly("num_leaves", &EquihashParams::num_leaves)
        .def_property_readonly("solution_indices", &EquihashParams::solution_indices)
        .def_property_readonly("solution_bytes", &EquihashParams::solution_bytes)
        .def_property_readonly("hash_bytes", &EquihashParams::hash_bytes)
        .def_property_readonly("personal", [](const EquihashParams& p) { u8 o[16]; p.personal(o); return py::bytes((char*)o, 16); });

    m.def("equihash_leaf", [](const EquihashParams& p, const py::bytes& input, u32 i) {
        std::string s = input;
        Blake2b base = equihash_base_state(p, reinterpret_cast<const u8*>(s.data()), s.size());
        u8 out[64];
        equihash_leaf(p, base, i, out);
        return py::bytes(reinterpret_cast<const char*>(out), size_t(p.hash_bytes()));
    });
    m.def("equihash_pack", [](const EquihashParams& p, const std::vector<u32>& idx) {
        Bytes b = equihash_pack_indices(p, idx);
        return py::bytes(reinterpret_cast<const char*>(b.data()), b.size());
    });
    m.def("equihash_unpack", [](const EquihashParams& p, const py::bytes& sol) {
        std::string s = sol;
        return equihash_unpack_indices(p, Bytes(s.begin(), s.end()));
    });
    m.def("equihash_verify", [](const EquihashParams& p, const py::bytes& input, const std::vector<u32>& idx) {
        std::string s = input;
        std::string reason;
        bool ok = equihash_verify(p, reinterpret_cast<const u8*>(s.data()), s.size(), idx, &reason);
        return py::make_tuple(ok, reason);
    });
    m.def("equihash_solve_cpu", [](const EquihashParams& p, const py::bytes& input, size_t max_solutions, int threads) {
        std::string s = input;
        EquihashSolveStats st;
        std::vector<std::vector<u32>> sols;
        {
            py::gil_scoped_release rel;
            sols = equihash_solve_cpu(p, reinterpret_cast<const u8*>(s.data()), s.size(), max_solutions, &st, threads);
        }
        py::dict stats;
        stats["rows_per_round"] = st.rows_per_round;
        stats["candidates"] = st.candidates;
        stats["discarded_duplicates"] = st.discarded_duplicates;
        return py::make_tuple(sols, stats);
    }, py::arg("params"), py::arg("input"), py::arg("max_solutions") = 64, py::arg("threads") = 0);
}
