// Bindings for the fee estimator (chain/fees.hpp).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../chain/fees.hpp"

namespace py = pybind11;
using namespace nodexa;

namespace {

Uint256 txid_of(const py::bytes& b) {
    std::string s = b;
    if (s.size() != 32) throw std::invalid_argument("expected a 32-byte txid");
    return Uint256::from_bytes(reinterpret_cast<const u8*>(s.data()));
}

py::dict range_dict(const FeeBucketRange& r) {
    py::dict d;
    d["startrange"] = r.start;
    d["endrange"] = r.end;
    d["withintarget"] = r.within_target;
    d["totalconfirmed"] = r.total_confirmed;
    d["inmempool"] = r.in_mempool;
    d["leftmempool"] = r.left_mempool;
    return d;
}

py::dict estimation_dict(const FeeEstimation& e) {
    py::dict d;
    d["pass"] = range_dict(e.pass);
    d["fail"] = range_dict(e.fail);
    d["decay"] = e.decay;
    d["scale"] = e.scale;
    return d;
}

FeeHorizon horizon_of(const std::string& s) {
    if (s == "short") return FeeHorizon::Short;
    if (s == "medium") return FeeHorizon::Medium;
    if (s == "long") return FeeHorizon::Long;
    throw std::invalid_argument("horizon must be short, medium or long");
}

}  // namespace

void bind_fees(py::module_& m) {
    py::class_<FeeEstimator>(m, "FeeEstimator")
        .def(py::init<>())
        .def("process_tx", [](FeeEstimator& f, const py::bytes& txid, u32 height, int64_t fee, int64_t vsize, bool valid) {
            f.process_tx(txid_of(txid), height, fee, vsize, valid);
        }, py::arg("txid"), py::arg("height"), py::arg("fee"), py::arg("vsize"), py::arg("valid") = true)
        .def("process_block", [](FeeEstimator& f, u32 height, const std::vector<py::bytes>& txids) {
            std::vector<Uint256> ids;
            ids.reserve(txids.size());
            for (const auto& t : txids) ids.push_back(txid_of(t));
            f.process_block(height, ids);
        })
        .def("remove_tx", [](FeeEstimator& f, const py::bytes& txid, bool in_block) {
            return f.remove_tx(txid_of(txid), in_block);
        }, py::arg("txid"), py::arg("in_block") = false)
        .def("flush_unconfirmed", &FeeEstimator::flush_unconfirmed)
        .def("estimate_fee", &FeeEstimator::estimate_fee)
        .def("estimate_raw_fee", [](const FeeEstimator& f, int target, double threshold, const std::string& h) {
            FeeEstimation e;
            const int64_t r = f.estimate_raw_fee(target, threshold, horizon_of(h), &e);
            return py::make_tuple(r, estimation_dict(e));
        })
        .def("estimate_smart_fee", [](const FeeEstimator& f, int target, bool conservative) {
            FeeEstimation e;
            FeeReason why = FeeReason::None;
            int returned = target;
            const int64_t r = f.estimate_smart_fee(target, conservative, &returned, &why, &e);
            return py::make_tuple(r, returned, std::string(fee_reason_string(why)), estimation_dict(e));
        }, py::arg("target"), py::arg("conservative") = true)
        .def("highest_target_tracked", [](const FeeEstimator& f, const std::string& h) {
            return f.highest_target_tracked(horizon_of(h));
        })
        .def("max_usable_estimate", &FeeEstimator::max_usable_estimate)
        .def("serialize", [](const FeeEstimator& f) {
            Bytes b = f.serialize();
            return py::bytes(reinterpret_cast<const char*>(b.data()), b.size());
        })
        .def("deserialize", [](FeeEstimator& f, const py::bytes& b) {
            std::string s = b, err;
            const bool ok = f.deserialize(Bytes(s.begin(), s.end()), &err);
            return py::make_tuple(ok, err);
        })
        .def_property_readonly("tracked", &FeeEstimator::tracked)
        .def_property_readonly("best_seen_height", &FeeEstimator::best_seen_height);
}
