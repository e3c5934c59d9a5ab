// Bindings for the consensus layer (chain/*), X16R and Equihash.
#include <pybind11/pybind11.h>

#include "../crypto/aes.hpp"
#include <pybind11/stl.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "../chain/headerbatch.hpp"
#include "../util/workpool.hpp"
#include "../chain/headerchain.hpp"
#include "../chain/script.hpp"
#include "../chain/validation.hpp"
#include "../pow/equihash.hpp"
#include "../crypto/hashes.hpp"
#include "../pow/legacy_algos.hpp"
#include "../pow/x16r.hpp"
#include "../pow/x16r_prims.hpp"
#include "../pow/kawpow.hpp"

namespace py = pybind11;
using namespace nodexa;

namespace {

Uint256 u256(const py::bytes& b) {
    std::string s = b;
    if (s.size() != 32) throw std::invalid_argument("expected 32 bytes");
    return Uint256::from_bytes(reinterpret_cast<const u8*>(s.data()));
}
py::bytes pyb(const Uint256& u) { return py::bytes(reinterpret_cast<const char*>(u.data), 32); }
py::bytes pyb(const Bytes& b) { return py::bytes(reinterpret_cast<const char*>(b.data()), b.size()); }
Bytes bytes_of(const py::bytes& b) { std::string s = b; return Bytes(s.begin(), s.end()); }

py::int_ arith_to_int(const ArithU256& a) {
    return py::int_(py::reinterpret_steal<py::object>(
        PyLong_FromString(const_cast<char*>(a.hex().c_str()), nullptr, 16)));
}
ArithU256 int_to_arith(const py::int_& v) {
    py::object mask = py::int_(1).attr("__lshift__")(256).attr("__sub__")(1);
    py::int_ x = v.attr("__and__")(mask);
    std::string hex = py::str(py::module_::import("builtins").attr("format")(x, "064x"));
    return ArithU256::from_uint256(Uint256::from_hex(hex));
}

}  // namespace

void bind_extra(py::module_& m) {
    m.attr("EQUIHASH_VERSION_BIT") = kEquihashVersionBit;

    // The constants the GPU DarkGravityWave kernel (hip/kernels/dgw.hip) needs, from the params.
    m.def("dgw_constants", [](const ChainParams& p) {
        const ConsensusParams& c = p.consensus;
        const Uint256 eq = c.equihash_limit.is_null() ? c.pow_limit : c.equihash_limit;
        std::vector<u32> limits;
        for (const Uint256* u : {&c.pow_limit, &c.kawpow_limit, &eq})
            for (int i = 0; i < 8; ++i) limits.push_back(load_le32(u->data + 4 * i));
        std::vector<u32> compacts = {ArithU256::from_uint256(c.pow_limit).get_compact(),
                                     ArithU256::from_uint256(c.kawpow_limit).get_compact(),
                                     ArithU256::from_uint256(eq).get_compact()};
        py::dict d;
        d["dgw_activation_block"] = p.dgw_activation_block;
        d["kawpow_time"] = p.kawpow_activation_time;
        d["equihash_time"] = p.equihash_activation_time;
        d["limits"] = limits;
        d["compacts"] = compacts;
        d["target_timespan"] = u32(kDgwPastBlocks * c.pow_target_spacing);
        return d;
    });

    // ------------------------------------------------ batch header verification (models/verify.py)
    // One pass over a header batch: for every KawPow header the 48-byte job record the GPU
    // verify kernels read (header hash progpow order, nonce64, height), its claimed mix and
    // nBits boundary (progpow / big-endian order) and the mix-only final hash that lets a
    // header whose claimed mix cannot meet nBits be rejected before any DAG access
    // (kawpow::verify's first check). kind: 0 = needs the full hash, 1 = high-hash already,
    // 2 = Equihash header, 3 = pre-KawPow (X16R) header.
    m.def("kawpow_batch_prepare", [](const py::list& headers, u32 kawpow_activation_time) {
        const size_t n = headers.size();
        std::vector<const BlockHeader*> hs(n);
        for (size_t i = 0; i < n; ++i) hs[i] = &headers[i].cast<const BlockHeader&>();
        std::string kinds(n, '\0'), jobs(n * 48, '\0'), mix(n * 32, '\0'), bound(n * 32, '\0'), pre(n * 32, '\0');
        {
            py::gil_scoped_release rel;
            auto one = [&](size_t i) {
                const BlockHeader& h = *hs[i];
                if (h.is_equihash()) { kinds[i] = 2; return; }
                if (!h.is_kawpow(kawpow_activation_time)) { kinds[i] = 3; return; }
                const Hash256 hh = h.kawpow_header_hash().to_progpow();
                const Hash256 mx = h.mix_hash.to_progpow();
                bool neg = false, ovf = false;
                ArithU256 t;
                t.set_compact(h.bits, &neg, &ovf);
                Hash256 b;  // zero boundary (nothing passes) for a negative / overflowing nBits
                if (!neg && !ovf) b = t.to_uint256().to_progpow();
                const Hash256 fin = kawpow_hash_no_verify(int(h.height), hh, mx, h.nonce64);
                kinds[i] = hash_le(fin, b) ? 0 : 1;
                char* j = jobs.data() + 48 * i;
                std::memcpy(j, hh.bytes, 32);
                store_le64(reinterpret_cast<u8*>(j + 32), h.nonce64);
                store_le32(reinterpret_cast<u8*>(j + 40), h.height);
                std::memcpy(mix.data() + 32 * i, mx.bytes, 32);
                std::memcpy(bound.data() + 32 * i, b.bytes, 32);
                std::memcpy(pre.data() + 32 * i, fin.bytes, 32);
            };
            const size_t threads = n >= 1024 ? std::min<size_t>(8, std::max(1u, std::thread::hardware_concurrency())) : 1;
            std::vector<std::thread> pool;
            const size_t step = (n + threads - 1) / threads;
            for (size_t t = 1; t < threads; ++t)
                pool.emplace_back([&, t] { for (size_t i = t * step; i < std::min(n, (t + 1) * step); ++i) one(i); });
            for (size_t i = 0; i < std::min(n, step); ++i) one(i);
            for (auto& th : pool) th.join();
        }
        return py::make_tuple(py::bytes(kinds), py::bytes(jobs), py::bytes(mix), py::bytes(bound), py::bytes(pre));
    }, py::arg("headers"), py::arg("kawpow_activation_time"));
    // The GPU form of the pass above (hip sha256d.hip: kawpow_mixonly_batch): only the header
    // kinds and the raw 120-byte KawPow headers are made on the host; SHA256d, both keccak-f800
    // absorbs and the nBits boundary run on the device. kind: 0 = KawPow, 2 = Equihash, 3 = X16R.
    m.def("kawpow_batch_headers", [](const py::list& headers, u32 kawpow_activation_time) {
        const size_t n = headers.size();
        std::string kinds(n, '\0'), raw(n * 120, '\0');
        for (size_t i = 0; i < n; ++i) {
            const BlockHeader& h = headers[i].cast<const BlockHeader&>();
            if (h.is_equihash()) { kinds[i] = 2; continue; }
            if (!h.is_kawpow(kawpow_activation_time)) { kinds[i] = 3; continue; }
            const Bytes b = h.bytes(kawpow_activation_time);
            if (b.size() != 120) throw std::runtime_error("KawPow header does not serialize to 120 bytes");
            std::memcpy(raw.data() + 120 * i, b.data(), 120);
        }
        return py::make_tuple(py::bytes(kinds), py::bytes(raw));
    }, py::arg("headers"), py::arg("kawpow_activation_time"));
    m.def("kawpow_programs_bytes", [](const std::vector<u64>& periods) {
        std::string out(periods.size() * 256, '\0');
        {
            py::gil_scoped_release rel;
            for (size_t k = 0; k < periods.size(); ++k) {
                const std::vector<u32> w = kawpow_program_words(make_kawpow_program(periods[k]));
                if (w.size() != 64) throw std::runtime_error("unexpected program size");
                std::memcpy(out.data() + 256 * k, w.data(), 256);
            }
        }
        return py::bytes(out);
    }, "64 little-endian u32 program words per period, concatenated (kawpow_program_words)");
    // ------------------------------------------------ uint256 / arith
    m.def("u256_hex", [](const py::bytes& b) { return u256(b).hex(); }, "uint256::GetHex of storage bytes");
    m.def("u256_from_hex", [](const std::string& s) { return pyb(Uint256::from_hex(s)); }, "uint256S");
    m.def("set_compact", [](u32 c) {
        bool neg = false, ovf = false;
        ArithU256 a;
        a.set_compact(c, &neg, &ovf);
        return py::make_tuple(arith_to_int(a), neg, ovf);
    });
    m.def("get_compact", [](const py::int_& v, bool negative) { return int_to_arith(v).get_compact(negative); },
          py::arg("value"), py::arg("negative") = false);
    m.def("arith_div", [](const py::int_& a, const py::int_& b) { return arith_to_int(int_to_arith(a) / int_to_arith(b)); });
    m.def("arith_mul", [](const py::int_& a, const py::int_& b) { return arith_to_int(int_to_arith(a) * int_to_arith(b)); });

    // ------------------------------------------------ auxiliary hashes (P20)
    m.def("sha1", [](const py::bytes& d) {
        std::string s = d;
        u8 o[20];
        sha1(reinterpret_cast<const u8*>(s.data()), s.size(), o);
        return py::bytes(reinterpret_cast<const char*>(o), 20);
    });
    m.def("hmac_sha256", [](const py::bytes& k, const py::bytes& d) {
        std::string ks = k, s = d;
        u8 o[32];
        hmac_sha256(reinterpret_cast<const u8*>(ks.data()), ks.size(), reinterpret_cast<const u8*>(s.data()), s.size(), o);
        return py::bytes(reinterpret_cast<const char*>(o), 32);
    });
    m.def("hmac_sha512", [](const py::bytes& k, const py::bytes& d) {
        std::string ks = k, s = d;
        u8 o[64];
        hmac_sha512(reinterpret_cast<const u8*>(ks.data()), ks.size(), reinterpret_cast<const u8*>(s.data()), s.size(), o);
        return py::bytes(reinterpret_cast<const char*>(o), 64);
    });
    m.def("siphash24", [](u64 k0, u64 k1, const py::bytes& d) {
        std::string s = d;
        return siphash24(k0, k1, reinterpret_cast<const u8*>(s.data()), s.size());
    });
    m.def("siphash_uint256", [](u64 k0, u64 k1, const py::bytes& v) { return siphash_uint256(k0, k1, u256(v).data); });
    m.def("siphash_uint256_extra", [](u64 k0, u64 k1, const py::bytes& v, u32 e) {
        return siphash_uint256_extra(k0, k1, u256(v).data, e);
    });
    m.def("murmur3_32", [](u32 seed, const py::bytes& d) {
        std::string s = d;
        return murmur3_32(seed, reinterpret_cast<const u8*>(s.data()), s.size());
    });
    m.def("aes256_cbc_encrypt", [](const py::bytes& key, const py::bytes& iv, const py::bytes& plain) {
        const std::string k = key, v = iv;
        if (k.size() != 32 || v.size() != 16) throw std::invalid_argument("key must be 32 bytes, iv 16");
        return pyb(aes256_cbc_encrypt(reinterpret_cast<const u8*>(k.data()), reinterpret_cast<const u8*>(v.data()),
                                      bytes_of(plain)));
    });
    m.def("aes256_cbc_decrypt", [](const py::bytes& key, const py::bytes& iv, const py::bytes& cipher) -> py::object {
        const std::string k = key, v = iv;
        if (k.size() != 32 || v.size() != 16) throw std::invalid_argument("key must be 32 bytes, iv 16");
        Bytes out;
        if (!aes256_cbc_decrypt(reinterpret_cast<const u8*>(k.data()), reinterpret_cast<const u8*>(v.data()),
                                bytes_of(cipher), out))
            return py::none();
        return pyb(out);
    });
    m.def("aes256_encrypt_block", [](const py::bytes& key, const py::bytes& block) {
        const std::string k = key, b = block;
        if (k.size() != 32 || b.size() != 16) throw std::invalid_argument("key 32 bytes, block 16");
        u8 out[16];
        Aes256(reinterpret_cast<const u8*>(k.data())).encrypt_block(reinterpret_cast<const u8*>(b.data()), out);
        return py::bytes(reinterpret_cast<const char*>(out), 16);
    });
    m.def("bytes_to_key_sha512", [](const std::string& pass, const py::bytes& salt, int rounds) {
        u8 k[32], v[16];
        bytes_to_key_sha512(pass, bytes_of(salt), rounds, k, v);
        return py::make_tuple(py::bytes(reinterpret_cast<const char*>(k), 32), py::bytes(reinterpret_cast<const char*>(v), 16));
    });
    m.def("sha512", [](const py::bytes& d) {
        std::string s = d;
        Hash512 h = sha512_hash(reinterpret_cast<const u8*>(s.data()), s.size());
        return py::bytes(reinterpret_cast<const char*>(h.bytes), 64);
    });

    // ------------------------------------------------ X16R
    m.def("x16r", [](const py::bytes& data, const py::bytes& prev) {
        std::string s = data;
        Uint256 p = u256(prev), out;
        {
            py::gil_scoped_release nogil;
            x16r_hash(reinterpret_cast<const u8*>(s.data()), s.size(), p.data, false, out.data);
        }
        return pyb(out);
    });
    m.def("x16rv2", [](const py::bytes& data, const py::bytes& prev) {
        std::string s = data;
        Uint256 p = u256(prev), out;
        {
            py::gil_scoped_release nogil;
            x16r_hash(reinterpret_cast<const u8*>(s.data()), s.size(), p.data, true, out.data);
        }
        return pyb(out);
    });
    m.def("x16r_algo", [](int algo, const py::bytes& data) {
        std::string s = data;
        Hash512 h = x16r_single(algo, reinterpret_cast<const u8*>(s.data()), s.size());
        return py::bytes(reinterpret_cast<const char*>(h.bytes), 64);
    });
    m.def("x16r_slot_available", &x16r_slot_available);
    m.def("x16r_groups", [](const py::buffer& headers) {
        // ops/x16r.x16r_hash_batch's launch tables: for each of the 16 steps, the headers grouped
        // by the slot they run there (a stable counting sort on the step's hashPrevBlock nibble,
        // GetHashSelection: nibble 48 + step = header byte 4 + (15 - step) / 2) as int32 bytes
        // (16 x n), and each step's 17 group offsets
        const py::buffer_info b = headers.request();
        const size_t len = size_t(b.size * b.itemsize);
        if (len % 80) throw std::invalid_argument("x16r_groups: 80-byte headers");
        const size_t n = len / 80;
        if (n > size_t(INT32_MAX)) throw std::invalid_argument("x16r_groups: too many headers");
        const u8* h = static_cast<const u8*>(b.ptr);
        std::string order(16 * n * 4, '\0');
        std::vector<int32_t> offsets(16 * 17, 0);
        {
            py::gil_scoped_release rel;
            int32_t* ord = reinterpret_cast<int32_t*>(order.data());
            parallel_for_each(16, [&](size_t s) {
                const size_t j = 15 - s, at = 4 + j / 2;
                const bool high = j & 1;
                int32_t* off = &offsets[s * 17];
                for (size_t i = 0; i < n; ++i) {
                    const u8 v = h[i * 80 + at];
                    ++off[1 + (high ? v >> 4 : v & 15)];
                }
                for (int k = 0; k < 16; ++k) off[k + 1] += off[k];
                int32_t pos[16];
                std::memcpy(pos, off, sizeof(pos));
                int32_t* o = ord + s * n;
                for (size_t i = 0; i < n; ++i) {
                    const u8 v = h[i * 80 + at];
                    o[pos[high ? v >> 4 : v & 15]++] = int32_t(i);
                }
            }, 1);
        }
        return py::make_tuple(py::bytes(order), offsets);
    }, py::arg("headers"));

    // ------------------------------------------------ HAVAL / Lyra2 (linked by the reference, unused by consensus)
    m.def("haval", [](const py::bytes& data, int passes, int out_bits) {
        std::string s = data;
        std::vector<u8> h = haval_hash(reinterpret_cast<const u8*>(s.data()), s.size(), passes, out_bits);
        return py::bytes(reinterpret_cast<const char*>(h.data()), h.size());
    }, py::arg("data"), py::arg("passes") = 3, py::arg("out_bits") = 256);
    m.def("gost", [](const py::bytes& data, int out_bits) {
        const std::string s = data;
        std::vector<u8> h = gost_streebog(reinterpret_cast<const u8*>(s.data()), s.size(), out_bits);
        return py::bytes(reinterpret_cast<const char*>(h.data()), h.size());
    }, py::arg("data"), py::arg("out_bits") = 512,
       "GOST R 34.11-2012 (Streebog), the reference's sph_gost256/512 byte conventions");
    m.def("lyra2", [](const py::bytes& pwd, const py::bytes& salt, u64 klen, u64 time_cost, u64 n_rows, u64 n_cols,
                      bool old_absorb) {
        std::string p = pwd, s = salt;
        std::vector<u8> k;
        {
            py::gil_scoped_release nogil;
            k = lyra2_hash(reinterpret_cast<const u8*>(p.data()), p.size(), reinterpret_cast<const u8*>(s.data()),
                           s.size(), klen, time_cost, n_rows, n_cols, old_absorb);
        }
        if (k.empty() && klen) throw std::invalid_argument("lyra2: nRows must be a power of two >= 4, input must fit the matrix");
        return py::bytes(reinterpret_cast<const char*>(k.data()), k.size());
    }, py::arg("pwd"), py::arg("salt"), py::arg("klen") = 32, py::arg("time_cost") = 1, py::arg("n_rows") = 4,
       py::arg("n_cols") = 4, py::arg("old_absorb") = false);
    m.def("x16r_search", [](const py::bytes& header80, bool v2, const py::bytes& target, u32 start, u64 count,
                            int threads) -> py::object {
        std::string h = header80;
        if (h.size() != 80) throw std::invalid_argument("x16r_search needs the 80-byte legacy header");
        Uint256 t = u256(target);
        X16rSearchResult r;
        {
            py::gil_scoped_release nogil;
            r = x16r_search(reinterpret_cast<const u8*>(h.data()), v2, t.data, start, count, threads);
        }
        if (!r.found) return py::make_tuple(py::none(), r.hashes);
        return py::make_tuple(py::make_tuple(r.nonce, py::bytes(reinterpret_cast<const char*>(r.hash), 32)), r.hashes);
    }, py::arg("header80"), py::arg("v2"), py::arg("target"), py::arg("start"), py::arg("count"),
       py::arg("threads") = 0,
       "lowest nNonce in [start, start+count) with X16R(V2) hash <= target (storage order) -> ((nonce, hash)|None, hashes)");
    m.def("x16r_selection", [](const py::bytes& prev, int i) { return x16r_selection(u256(prev).data, i); });

    // ------------------------------------------------ script / addresses
    m.def("base58check_encode", [](const py::bytes& p) { return base58check_encode(bytes_of(p)); });
    m.def("base58check_decode", [](const std::string& s) -> py::object {
        Bytes out;
        if (!base58check_decode(s, out)) return py::none();
        return pyb(out);
    });
    m.def("address_to_script", [](const std::string& a, u8 pkh, u8 sh) -> py::object {
        Bytes s;
        if (!address_to_script(a, pkh, sh, s)) return py::none();
        return pyb(s);
    });
    m.def("script_to_address", [](const py::bytes& s, u8 pkh, u8 sh) { return script_to_address(bytes_of(s), pkh, sh); });
    m.def("script_push_int", [](int64_t v) { return pyb(ScriptBuilder().push_int(v).s); });
    m.def("script_push_data", [](const py::bytes& d) { return pyb(ScriptBuilder().push_data(bytes_of(d)).s); });
    m.def("scriptnum", [](int64_t v) { return pyb(ScriptBuilder::scriptnum(v)); });
    m.def("ripemd160", [](const py::bytes& d) { Bytes b = bytes_of(d); u8 o[20]; ripemd160(b.data(), b.size(), o); return py::bytes((char*)o, 20); });
    m.def("hash160", [](const py::bytes& d) { Bytes b = bytes_of(d); u8 o[20]; hash160(b.data(), b.size(), o); return py::bytes((char*)o, 20); });

    // ------------------------------------------------ transactions / blocks
    py::class_<OutPoint>(m, "OutPoint")
        .def(py::init<>())
        .def_property("hash", [](const OutPoint& o) { return pyb(o.hash); }, [](OutPoint& o, const py::bytes& b) { o.hash = u256(b); })
        .def_readwrite("n", &OutPoint::n)
        .def("is_null", &OutPoint::is_null);
    py::class_<TxIn>(m, "TxIn")
        .def(py::init<>())
        .def_readwrite("prevout", &TxIn::prevout)
        .def_property("script_sig", [](const TxIn& t) { return pyb(t.script_sig); }, [](TxIn& t, const py::bytes& b) { t.script_sig = bytes_of(b); })
        .def_readwrite("sequence", &TxIn::sequence)
        .def_property("witness", [](const TxIn& t) { py::list l; for (auto& w : t.witness) l.append(pyb(w)); return l; },
                      [](TxIn& t, const std::vector<py::bytes>& w) { t.witness.clear(); for (auto& x : w) t.witness.push_back(bytes_of(x)); });
    py::class_<TxOut>(m, "TxOut")
        .def(py::init<>())
        .def(py::init([](Amount v, const py::bytes& s) { TxOut o; o.value = v; o.script_pubkey = bytes_of(s); return o; }))
        .def_readwrite("value", &TxOut::value)
        .def_property("script_pubkey", [](const TxOut& t) { return pyb(t.script_pubkey); }, [](TxOut& t, const py::bytes& b) { t.script_pubkey = bytes_of(b); });
    py::class_<Transaction>(m, "Transaction")
        .def(py::init<>())
        .def_readwrite("version", &Transaction::version)
        .def_readwrite("vin", &Transaction::vin)
        .def_readwrite("vout", &Transaction::vout)
        .def_readwrite("lock_time", &Transaction::lock_time)
        .def("serialize", [](const Transaction& t, bool w) { return pyb(t.bytes(w)); }, py::arg("with_witness") = true)
        .def_static("deserialize", [](const py::bytes& b, bool allow_witness) {
            Bytes d = bytes_of(b);
            Reader r(d);
            Transaction t = Transaction::deserialize(r, allow_witness);
            if (!r.empty()) throw std::runtime_error("trailing bytes after transaction");
            return t;
        }, py::arg("data"), py::arg("allow_witness") = true)
        .def_static("deserialize_prefix", [](const py::bytes& b, size_t offset) {
            Bytes d = bytes_of(b);
            if (offset > d.size()) throw std::out_of_range("offset past the end");
            Reader r(d.data() + offset, d.size() - offset);
            Transaction t = Transaction::deserialize(r);
            return py::make_tuple(t, r.pos());
        }, py::arg("data"), py::arg("offset") = 0, "(tx, bytes consumed) for a transaction at data[offset:]")
        .def("txid", [](const Transaction& t) { return pyb(t.txid()); })
        .def("wtxid", [](const Transaction& t) { return pyb(t.wtxid()); })
        .def("is_coinbase", &Transaction::is_coinbase)
        .def("has_witness", &Transaction::has_witness)
        .def("value_out", &Transaction::value_out);
    py::class_<BlockHeader>(m, "BlockHeader")
        .def(py::init<>())
        .def_readwrite("version", &BlockHeader::version)
        .def_property("prev", [](const BlockHeader& h) { return pyb(h.prev); }, [](BlockHeader& h, const py::bytes& b) { h.prev = u256(b); })
        .def_property("merkle_root", [](const BlockHeader& h) { return pyb(h.merkle_root); }, [](BlockHeader& h, const py::bytes& b) { h.merkle_root = u256(b); })
        .def_readwrite("time", &BlockHeader::time)
        .def_readwrite("bits", &BlockHeader::bits)
        .def_readwrite("nonce", &BlockHeader::nonce)
        .def_readwrite("height", &BlockHeader::height)
        .def_readwrite("nonce64", &BlockHeader::nonce64)
        .def_property("mix_hash", [](const BlockHeader& h) { return pyb(h.mix_hash); }, [](BlockHeader& h, const py::bytes& b) { h.mix_hash = u256(b); })
        .def_property("nonce256", [](const BlockHeader& h) { return pyb(h.nonce256); }, [](BlockHeader& h, const py::bytes& b) { h.nonce256 = u256(b); })
        .def_property("solution", [](const BlockHeader& h) { return py::bytes(reinterpret_cast<const char*>(h.solution.data()), h.solution.size()); },
                      [](BlockHeader& h, const py::bytes& b) { h.solution = bytes_of(b); })
        .def("is_equihash", &BlockHeader::is_equihash)
        .def("equihash_input", [](const BlockHeader& h) { Bytes b = h.equihash_input(); return py::bytes(reinterpret_cast<const char*>(b.data()), b.size()); })
        .def("equihash_hash", [](const BlockHeader& h, u32 act) { return pyb(h.equihash_hash(act)); })
        .def("kawpow_input", [](const BlockHeader& h) { Bytes b = h.kawpow_input(); return py::bytes(reinterpret_cast<const char*>(b.data()), b.size()); })
        .def("serialize", [](const BlockHeader& h, u32 act) { return pyb(h.bytes(act)); })
        .def_static("deserialize", [](const py::bytes& b, u32 act) { Bytes d = bytes_of(b); Reader r(d); return BlockHeader::deserialize(r, act); })
        .def_static("deserialize_prefix", [](const py::bytes& b, u32 act, size_t off) {
            Bytes d = bytes_of(b);
            if (off > d.size()) throw std::out_of_range("offset past the end");
            Reader r(d.data() + off, d.size() - off);
            BlockHeader h = BlockHeader::deserialize(r, act);
            return py::make_tuple(h, r.pos());
        }, py::arg("data"), py::arg("act"), py::arg("offset") = 0, "(header, bytes used) from a prefix")
        .def("kawpow_header_hash", [](const BlockHeader& h) { return pyb(h.kawpow_header_hash()); })
        .def("legacy80", [](const BlockHeader& h) { return pyb(h.legacy80()); });
    m.def("deserialize_headers", [](const py::bytes& b, u32 act) {
        // concatenated headers of mixed formats (80 / 120 / Equihash-extended)
        Bytes d = bytes_of(b);
        Reader r(d);
        std::vector<BlockHeader> out;
        while (!r.empty()) out.push_back(BlockHeader::deserialize(r, act));
        return out;
    });
    // P2P `headers` message payload: compact-size count, then header || compact-size(0)
    // per entry (src/net_processing.cpp:2166-2187; <= MAX_HEADERS_RESULTS = 2000).
    m.def("headers_msg_decode", [](const py::bytes& b, u32 act) {
        Bytes d = bytes_of(b);
        Reader r(d);
        const u64 n = r.compact_size();
        if (n > 2000) throw std::invalid_argument("headers message with more than 2000 headers");
        std::vector<BlockHeader> out;
        out.reserve(size_t(n));
        for (u64 i = 0; i < n; ++i) {
            out.push_back(BlockHeader::deserialize(r, act));
            if (r.compact_size() != 0) throw std::invalid_argument("headers message: non-zero tx count");
        }
        return out;
    });
    m.def("headers_msg_encode", [](const std::vector<BlockHeader>& hs, u32 act) {
        Writer w;
        w.compact_size(hs.size());
        for (auto& h : hs) {
            w.raw(h.bytes(act));
            w.compact_size(0);
        }
        return pyb(w.buf);
    });
    py::class_<Block>(m, "Block")
        .def(py::init<>())
        .def_readwrite("header", &Block::header)
        .def_readwrite("vtx", &Block::vtx)
        .def("serialize", [](const Block& b, u32 act, bool w) { return pyb(b.bytes(act, w)); }, py::arg("act"), py::arg("with_witness") = true)
        .def_static("deserialize", [](const py::bytes& b, u32 act) {
            Bytes d = bytes_of(b);
            Reader r(d);
            Block blk = Block::deserialize(r, act);
            if (!r.empty()) throw std::runtime_error("trailing bytes after block");
            return blk;
        })
        .def("merkle_root", [](const Block& b) { bool mut = false; Uint256 r = block_merkle_root(b, &mut); return py::make_tuple(pyb(r), mut); })
        .def("witness_merkle_root", [](const Block& b) { return pyb(block_witness_merkle_root(b)); })
        .def("witness_commitment_index", [](const Block& b) { return witness_commitment_index(b); })
        .def("weight", &Block::weight)
        .def("total_size", &Block::total_size)
        .def("stripped_size", &Block::stripped_size);
    m.def("compute_merkle_root", [](const std::vector<py::bytes>& leaves) {
        std::vector<Uint256> l;
        for (auto& x : leaves) l.push_back(u256(x));
        bool mut = false;
        Uint256 r = compute_merkle_root(l, &mut);
        return py::make_tuple(pyb(r), mut);
    });

    // ------------------------------------------------ params / rules
    py::class_<ChainParams>(m, "ChainParams")
        .def_readonly("network_id", &ChainParams::network_id)
        .def_readonly("equihash_n", &ChainParams::equihash_n)
        .def_readonly("equihash_k", &ChainParams::equihash_k)
        .def_property_readonly("message_start", [](const ChainParams& p) { return py::bytes((const char*)p.message_start, 4); })
        .def_readonly("default_port", &ChainParams::default_port)
        .def_readonly("default_rpc_port", &ChainParams::default_rpc_port)
        .def_readonly("pubkey_prefix", &ChainParams::pubkey_prefix)
        .def_readonly("script_prefix", &ChainParams::script_prefix)
        .def_readwrite("genesis", &ChainParams::genesis)
        .def_property_readonly("genesis_hash", [](const ChainParams& p) { return pyb(p.consensus.genesis_hash); })
        .def_property_readonly("pow_limit", [](const ChainParams& p) { return pyb(p.consensus.pow_limit); })
        .def_property_readonly("last_checkpoint_height", &ChainParams::last_checkpoint_height)
        .def_property_readonly("kawpow_limit", [](const ChainParams& p) { return pyb(p.consensus.kawpow_limit); })
        .def_property("equihash_limit", [](const ChainParams& p) { return pyb(p.consensus.equihash_limit); },
                      [](ChainParams& p, const py::bytes& b) { p.consensus.equihash_limit = u256(b); })
        .def_property_readonly("pow_target_spacing", [](const ChainParams& p) { return p.consensus.pow_target_spacing; })
        .def_property_readonly("pow_allow_min_difficulty_blocks", [](const ChainParams& p) { return p.consensus.pow_allow_min_difficulty_blocks; })
        .def_property_readonly("checkpoints", [](const ChainParams& p) { py::dict d; for (auto& kv : p.checkpoints) d[py::int_(kv.first)] = pyb(kv.second); return d; })
        .def("clear_checkpoints", [](ChainParams& p) { p.checkpoints.clear(); })  // -checkpoints=0
        .def_readwrite("community_autonomous_pct", &ChainParams::community_autonomous_pct)
        .def_readwrite("community_autonomous_address", &ChainParams::community_autonomous_address)
        .def_readwrite("dgw_activation_block", &ChainParams::dgw_activation_block)
        .def_readwrite("kawpow_activation_time", &ChainParams::kawpow_activation_time)
        .def_readwrite("x16rv2_activation_time", &ChainParams::x16rv2_activation_time)
        .def_readwrite("equihash_activation_time", &ChainParams::equihash_activation_time)
        .def_readwrite("max_reorg_depth", &ChainParams::max_reorg_depth)
        .def_readwrite("min_reorg_peers", &ChainParams::min_reorg_peers)
        .def_readwrite("min_reorg_age", &ChainParams::min_reorg_age)
        .def_readonly("mine_blocks_on_demand", &ChainParams::mine_blocks_on_demand)
        .def_readonly("mining_requires_peers", &ChainParams::mining_requires_peers);
    m.def("make_chain_params", &make_chain_params);
    m.def("check_proof_of_work", [](const py::bytes& h, u32 bits, const ChainParams& p) { return check_proof_of_work(u256(h), bits, p); });
    m.def("block_proof", [](u32 bits) { return arith_to_int(block_proof(bits)); });
    m.def("block_subsidy", &block_subsidy);
    m.def("difficulty_from_bits", &difficulty_from_bits);

    py::class_<HeaderIndex>(m, "HeaderIndex")
        .def_property_readonly("hash", [](const HeaderIndex& i) { return pyb(i.hash); })
        .def_readonly("height", &HeaderIndex::height)
        .def_readonly("time", &HeaderIndex::time)
        .def_readonly("bits", &HeaderIndex::bits)
        .def_readonly("header", &HeaderIndex::header)
        .def_property_readonly("chain_work", [](const HeaderIndex& i) { return arith_to_int(i.chain_work); })
        .def_property_readonly("prev_hash", [](const HeaderIndex& i) { return i.prev ? pyb(i.prev->hash) : pyb(Uint256()); })
        .def_property_readonly("skip_height", [](const HeaderIndex& i) { return i.skip ? i.skip->height : -1; })
        .def("ancestor", &HeaderIndex::ancestor, py::return_value_policy::reference_internal)
        .def("median_time_past", &HeaderIndex::median_time_past);

    py::class_<AcceptResult>(m, "AcceptResult")
        .def_readonly("ok", &AcceptResult::ok)
        .def_readonly("duplicate", &AcceptResult::duplicate)
        .def_readonly("reject", &AcceptResult::reject)
        .def_readonly("dos", &AcceptResult::dos)
        .def_property_readonly("index", [](const AcceptResult& r) { return r.index; }, py::return_value_policy::reference);

    // ------------------------------------------------ HeaderBatch (models/verify.py resident pipeline)
    static_assert(sizeof(Uint256) == 32, "hash blobs are read as Uint256 arrays");
    auto view = [](const auto& s) {  // zero-copy, read-only: the batch must outlive it
        return py::memoryview::from_memory(const_cast<char*>(s.data()), py::ssize_t(s.size()), true);
    };
    m.def("copy_into", [](const py::buffer& dst, size_t offset, const py::buffer& src) {
        // dst[offset : offset + len(src)] = src on all cores (dst: a writable buffer such as the
        // numpy view of a pinned staging tensor; bounds checked): the resident verify stages its
        // 1.3 MB of rows in a fraction of a single-threaded copy
        const py::buffer_info db = dst.request(true), sb = src.request();
        const size_t dlen = size_t(db.size) * size_t(db.itemsize), len = size_t(sb.size) * size_t(sb.itemsize);
        if (offset > dlen || len > dlen - offset) throw std::out_of_range("copy_into: source does not fit");
        const char* s = static_cast<const char*>(sb.ptr);
        char* d = static_cast<char*>(db.ptr) + offset;
        constexpr size_t kChunk = 64 << 10;
        py::gil_scoped_release rel;
        if (len < 4 * kChunk) {
            std::memcpy(d, s, len);
            return;
        }
        parallel_for_each((len + kChunk - 1) / kChunk, [&](size_t c) {
            const size_t o = c * kChunk;
            std::memcpy(d + o, s + o, std::min(kChunk, len - o));
        }, 1);
    }, py::arg("dst"), py::arg("offset"), py::arg("src"));
    m.def("workpool_selftest", [](size_t n, int64_t throw_at) {
        // test hook: sum of 0..n-1 over the pool; the part holding index `throw_at` (if >= 0)
        // throws, which must reach the caller as an exception once every part has returned
        std::atomic<uint64_t> sum{0};
        {
            py::gil_scoped_release rel;
            parallel_for_range(n, [&](size_t lo, size_t hi) {
                uint64_t s = 0;
                for (size_t i = lo; i < hi; ++i) {
                    if (throw_at >= 0 && i == size_t(throw_at)) throw std::runtime_error("workpool_selftest: part failed");
                    s += i;
                }
                sum += s;
            }, 1);
        }
        return uint64_t(sum.load());
    }, py::arg("n"), py::arg("throw_at") = -1);
    m.def("copy_into_many", [](const py::buffer& dst, const py::list& parts) {
        // dst[offset : offset + len(src)] = src for every (offset, src) of `parts`, bounds checked
        // before anything is written; sources of 256 KiB or more are copied on all cores (the
        // resident verify stages its whole upload with this one call)
        const py::buffer_info db = dst.request(true);
        const size_t dlen = size_t(db.size) * size_t(db.itemsize);
        char* d = static_cast<char*>(db.ptr);
        std::vector<py::buffer_info> infos;
        std::vector<size_t> offs;
        infos.reserve(parts.size());
        for (const py::handle& item : parts) {
            const py::tuple t = item.cast<py::tuple>();
            if (t.size() != 2) throw std::invalid_argument("copy_into_many: (offset, buffer) pairs");
            const size_t o = t[0].cast<size_t>();
            py::buffer_info bi = t[1].cast<py::buffer>().request();
            const size_t len = size_t(bi.size) * size_t(bi.itemsize);
            if (o > dlen || len > dlen - o) throw std::out_of_range("copy_into_many: a source does not fit");
            offs.push_back(o);
            infos.push_back(std::move(bi));
        }
        py::gil_scoped_release rel;
        constexpr size_t kChunk = 64 << 10;
        for (size_t k = 0; k < infos.size(); ++k) {
            const char* src = static_cast<const char*>(infos[k].ptr);
            const size_t len = size_t(infos[k].size) * size_t(infos[k].itemsize);
            char* to = d + offs[k];
            if (len < 4 * kChunk) {
                if (len) std::memcpy(to, src, len);
                continue;
            }
            parallel_for_each((len + kChunk - 1) / kChunk, [&](size_t c) {
                const size_t o = c * kChunk;
                std::memcpy(to + o, src + o, std::min(kChunk, len - o));
            }, 1);
        }
    }, py::arg("dst"), py::arg("parts"));
    m.def("wave_slots", [](const py::buffer& kinds_buf, const py::buffer& heights_buf, size_t lo, size_t hi) {
        // kawpow_verify_waves' slot table for the KawPow rows (kind 0) of [lo, hi): the rows grouped
        // by ProgPoW period (height / 3), 4 slots per wave64 (one 16-lane group each), -1 = idle
        // group, values relative to lo; little-endian int32 bytes
        const py::buffer_info kb = kinds_buf.request(), hb = heights_buf.request();
        const u8* kinds = static_cast<const u8*>(kb.ptr);
        const u32* heights = static_cast<const u32*>(hb.ptr);
        const size_t n = std::min(size_t(kb.size * kb.itemsize), size_t(hb.size * hb.itemsize) / 4);
        hi = std::min(hi, n);
        std::vector<u32> rows;
        rows.reserve(hi > lo ? hi - lo : 0);
        bool sorted = true;
        for (size_t r = lo; r < hi; ++r) {
            if (kinds[r] != 0) continue;
            if (!rows.empty() && heights[r] / 3 < heights[rows.back()] / 3) sorted = false;
            rows.push_back(u32(r));
        }
        if (!sorted)
            std::stable_sort(rows.begin(), rows.end(), [&](u32 a, u32 b) { return heights[a] / 3 < heights[b] / 3; });
        std::vector<int32_t> out;
        out.reserve(rows.size() * 2 + 4);
        for (size_t i = 0; i < rows.size();) {
            const u32 per = heights[rows[i]] / 3;
            for (; i < rows.size() && heights[rows[i]] / 3 == per; ++i) out.push_back(int32_t(rows[i] - lo));
            while (out.size() % 4) out.push_back(-1);
        }
        return py::bytes(reinterpret_cast<const char*>(out.data()), out.size() * 4);
    }, py::arg("kinds"), py::arg("heights"), py::arg("lo"), py::arg("hi"));
    py::class_<HeaderBatch, std::shared_ptr<HeaderBatch>>(m, "HeaderBatch")
        .def_static("from_bytes", [](const py::buffer& buf, u32 act) {
            const py::buffer_info bi = buf.request();
            const u8* p = static_cast<const u8*>(bi.ptr);
            const size_t len = size_t(bi.size) * size_t(bi.itemsize);
            // an immutable bytes object is read in place by the deferred decode (the batch holds a
            // reference); any other buffer could change under it, so its records are copied
            std::shared_ptr<const void> keep;
            if (PyBytes_Check(buf.ptr())) {
                PyObject* o = buf.ptr();
                Py_INCREF(o);
                keep = std::shared_ptr<const void>(o, [](const void* q) {
                    if (!Py_IsInitialized()) return;  // interpreter shutdown: leave the reference
                    py::gil_scoped_acquire g;
                    Py_DECREF(reinterpret_cast<PyObject*>(const_cast<void*>(q)));
                });
            }
            py::gil_scoped_release rel;
            return std::make_shared<HeaderBatch>(HeaderBatch::from_bytes(p, len, act, std::move(keep)));
        }, py::arg("data"), py::arg("kawpow_activation_time"),
           "parse concatenated serialized headers (80 / 120 / Equihash-extended) and pack them")
        .def_static("from_headers", [](std::vector<BlockHeader> hs, u32 act) {
            py::gil_scoped_release rel;
            return std::make_shared<HeaderBatch>(HeaderBatch::from_headers(std::move(hs), act));
        }, py::arg("headers"), py::arg("kawpow_activation_time"))
        .def("__len__", &HeaderBatch::size)
        .def_readonly("kawpow_activation_time", &HeaderBatch::act)
        .def_property_readonly("kinds", [view](const HeaderBatch& b) { return view(b.kinds); })
        .def_property_readonly("rows", [view](const HeaderBatch& b) { return view(b.rows); })
        .def_property_readonly("eq_index", [](const HeaderBatch& b) {
            return py::memoryview::from_memory(const_cast<u32*>(b.eq_index.data()), py::ssize_t(b.eq_index.size() * 4),
                                               true);
        })
        .def_property_readonly("eq_msgs", [view](const HeaderBatch& b) { return view(b.eq_msgs); })
        .def_property_readonly("eq_sols", [view](const HeaderBatch& b) { return view(b.eq_sols); })
        .def_property_readonly("eq_ser", [view](const HeaderBatch& b) { return view(b.eq_ser); })
        .def_readonly("eq_ser_len", &HeaderBatch::eq_ser_len)
        .def_readonly("eq_uniform", &HeaderBatch::eq_uniform)
        .def("kawpow_plan", [](const HeaderBatch& b, u32 epoch_length) -> py::object {
            // the resident verify's plan in one pass: the (epoch, lo, hi) ranges of the KawPow
            // rows and every row's nHeight, nTime and nBits (row bytes 76, 68, 72; u32 bytes each);
            // None when the KawPow rows' epochs are not in ascending order
            if (epoch_length == 0) throw std::invalid_argument("epoch_length");
            const size_t n = b.size();
            std::string heights(n * 4, '\0'), times(n * 4, '\0'), bits(n * 4, '\0');
            py::list ranges;
            long long cur = -1;
            size_t lo = 0, hi = 0;
            bool ordered = true;
            for (size_t i = 0; i < n; ++i) {
                const u8* row = reinterpret_cast<const u8*>(b.rows.data()) + i * kBatchRow;
                const u32 h = load_le32(row + 76);
                std::memcpy(&heights[i * 4], row + 76, 4);
                std::memcpy(&times[i * 4], row + 68, 4);
                std::memcpy(&bits[i * 4], row + 72, 4);
                if (b.kinds[i] != 0 || !ordered) continue;
                const long long e = h / epoch_length;
                if (e < cur) {
                    ordered = false;
                } else if (e != cur) {
                    if (cur >= 0) ranges.append(py::make_tuple(cur, lo, hi));
                    cur = e;
                    lo = i;
                    hi = i + 1;
                } else {
                    hi = i + 1;
                }
            }
            if (!ordered) return py::none();
            if (cur >= 0) ranges.append(py::make_tuple(cur, lo, hi));
            return py::make_tuple(ranges, py::bytes(heights), py::bytes(times), py::bytes(bits));
        }, py::arg("epoch_length"))
        .def("materialize", [](HeaderBatch& b) {
            py::gil_scoped_release rel;
            b.materialize();
        }, "decode the wire records into header objects now (from_bytes defers it; every accessor "
           "below does it on first use)")
        .def("header", [](HeaderBatch& b, size_t i) {
            if (i >= b.size()) throw py::index_error();
            return b.header(i);  // one record decoded if the batch is not materialized yet
        })
        .def("headers", [](HeaderBatch& b, size_t lo, size_t hi) {
            {
                py::gil_scoped_release rel;
                b.materialize();
            }
            hi = std::min(hi, b.hs.size());
            return std::vector<BlockHeader>(b.hs.begin() + std::min(lo, hi), b.hs.begin() + hi);
        }, py::arg("lo") = 0, py::arg("hi") = size_t(-1));

    py::class_<AcceptPrep, std::shared_ptr<AcceptPrep>>(m, "AcceptPrep")
        .def_readonly("n", &AcceptPrep::n);
    py::class_<HeaderChain, std::shared_ptr<HeaderChain>>(m, "HeaderChain")
        .def("accept_batch",
             [](HeaderChain& c, HeaderBatch& b, int64_t adjusted_time, const py::object& hashes,
                const py::object& bits, size_t lo, size_t hi) {
                 {
                     py::gil_scoped_release rel;
                     b.materialize();
                 }
                 // accept_headers over batch headers [lo, hi) with the device pipeline's block hashes
                 // (n x 32, storage order) and DGW nBits (n x u32, 0 = host decides), both indexed
                 // by batch position: (accepted, reject reason or None, dos)
                 hi = std::min(hi, b.hs.size());
                 lo = std::min(lo, hi);
                 const Uint256* kh = nullptr;
                 const u32* kb = nullptr;
                 py::buffer_info hb, bb;
                 if (!hashes.is_none()) {
                     hb = hashes.cast<py::buffer>().request();
                     if (size_t(hb.size * hb.itemsize) != b.hs.size() * 32) throw std::invalid_argument("hashes: n x 32 bytes");
                     kh = reinterpret_cast<const Uint256*>(hb.ptr) + lo;
                 }
                 if (!bits.is_none()) {
                     bb = bits.cast<py::buffer>().request();
                     if (size_t(bb.size * bb.itemsize) != b.hs.size() * 4) throw std::invalid_argument("bits: n x 4 bytes");
                     kb = static_cast<const u32*>(bb.ptr) + lo;
                 }
                 std::vector<AcceptResult> r;
                 {
                     py::gil_scoped_release rel;
                     r = c.accept_headers(b.hs.data() + lo, hi - lo, adjusted_time, false, kh, kb);
                 }
                 size_t ok = 0;
                 while (ok < r.size() && r[ok].ok) ++ok;
                 py::object why = py::none();
                 int dos = 0;
                 if (ok < r.size()) {
                     why = py::str(r[ok].reject);
                     dos = r[ok].dos;
                 }
                 return py::make_tuple(ok, why, dos);
             },
             py::arg("batch"), py::arg("adjusted_time"), py::arg("hashes") = py::none(), py::arg("bits") = py::none(),
             py::arg("lo") = 0, py::arg("hi") = size_t(-1))
        .def("prepare_batch",
             [](const HeaderChain& c, HeaderBatch& b, int64_t adjusted_time, const py::buffer& hashes,
                const py::buffer& bits) {
                 // accept_batch's read-only first phase over the whole batch (hashes n x 32 and
                 // nBits n x u32 are copied): the result commits a prefix later (commit_batch)
                 {
                     py::gil_scoped_release rel;
                     b.materialize();
                 }
                 const py::buffer_info hb = hashes.request(), bb = bits.request();
                 const size_t n = b.hs.size();
                 if (size_t(hb.size * hb.itemsize) != n * 32) throw std::invalid_argument("hashes: n x 32 bytes");
                 if (size_t(bb.size * bb.itemsize) != n * 4) throw std::invalid_argument("bits: n x 4 bytes");
                 py::gil_scoped_release rel;
                 return std::make_shared<AcceptPrep>(c.prepare_headers(
                     b.hs.data(), n, adjusted_time, false, reinterpret_cast<const Uint256*>(hb.ptr),
                     static_cast<const u32*>(bb.ptr)));
             },
             py::arg("batch"), py::arg("adjusted_time"), py::arg("hashes"), py::arg("bits"),
             py::keep_alive<0, 2>())  // the prepared state points into the batch's headers
        .def("commit_batch",
             [](HeaderChain& c, AcceptPrep& p, size_t hi) {
                 // accept headers [0, hi) of a prepare_batch: (accepted, reject reason or None, dos)
                 std::vector<AcceptResult> r;
                 {
                     py::gil_scoped_release rel;
                     r = c.commit_headers(p, hi);
                 }
                 size_t ok = 0;
                 while (ok < r.size() && r[ok].ok) ++ok;
                 py::object why = py::none();
                 int dos = 0;
                 if (ok < r.size()) {
                     why = py::str(r[ok].reject);
                     dos = r[ok].dos;
                 }
                 return py::make_tuple(ok, why, dos);
             },
             py::arg("prepared"), py::arg("hi"))
        .def("dgw_ancestors",
             [](const HeaderChain& c, const py::bytes& prev) -> py::object {
                 // the DGW series prefix of a batch whose first header builds on `prev`: prev and up
                 // to 179 of its ancestors, oldest first -> (times, bits, a, base_height) or None
                 const HeaderIndex* base = c.find(u256(prev));
                 const ConsensusParams& cp = c.params().consensus;
                 if (base == nullptr || (cp.pow_allow_min_difficulty_blocks && cp.pow_no_retargeting)) return py::none();
                 std::vector<const HeaderIndex*> anc;
                 for (const HeaderIndex* q = base; q && anc.size() < size_t(kDgwPastBlocks); q = q->prev) anc.push_back(q);
                 const size_t a = anc.size();
                 std::vector<u32> times(a), bits(a);
                 for (size_t k = 0; k < a; ++k) {
                     times[k] = anc[a - 1 - k]->time;
                     bits[k] = anc[a - 1 - k]->bits;
                 }
                 return py::make_tuple(py::bytes(reinterpret_cast<const char*>(times.data()), a * 4),
                                       py::bytes(reinterpret_cast<const char*>(bits.data()), a * 4), a, base->height);
             }, py::arg("prev"))
        .def("dgw_series_batch",
             [](const HeaderChain& c, const HeaderBatch& b, const py::buffer& hashes, size_t lo, size_t hi) -> py::object {
                 hi = std::min(hi, b.hs.size());
                 lo = std::min(lo, hi);
                 const py::buffer_info hb = hashes.request();
                 if (size_t(hb.size * hb.itemsize) != b.hs.size() * 32) throw std::invalid_argument("hashes: n x 32 bytes");
                 std::vector<u32> times, bits;
                 size_t a = 0;
                 int base = 0;
                 if (!c.dgw_series(b.hs.data() + lo, hi - lo, reinterpret_cast<const Uint256*>(hb.ptr) + lo, times, bits,
                                   a, base))
                     return py::none();
                 return py::make_tuple(py::bytes(reinterpret_cast<const char*>(times.data()), times.size() * 4),
                                       py::bytes(reinterpret_cast<const char*>(bits.data()), bits.size() * 4), a, base);
             },
             py::arg("batch"), py::arg("hashes"), py::arg("lo") = 0, py::arg("hi") = size_t(-1))
        .def(py::init([](const ChainParams& p) { return std::make_shared<HeaderChain>(p, std::make_shared<CpuPowVerifier>()); }))
        .def_property_readonly("params", &HeaderChain::params, py::return_value_policy::reference_internal)
        .def("set_kawpow_activation_time", [](HeaderChain& c, u32 t) { c.mutable_params().kawpow_activation_time = t; })
        .def("add_anchor",
             [](HeaderChain& c, const std::vector<BlockHeader>& hs, int base_height, const py::int_& base_work) {
                 return c.add_anchor(hs, base_height, int_to_arith(base_work));
             },
             py::arg("headers"), py::arg("base_height"), py::arg("base_work"), py::return_value_policy::reference_internal)
        .def_readwrite("strict_kawpow_height", &HeaderChain::strict_kawpow_height)
        .def_readwrite("max_reorg_depth", &HeaderChain::max_reorg_depth)
        .def("check_header", &HeaderChain::check_header, py::call_guard<py::gil_scoped_release>())
        .def("accept_header", &HeaderChain::accept_header, py::arg("header"), py::arg("adjusted_time"), py::arg("check_pow") = true,
             py::call_guard<py::gil_scoped_release>())
        .def("accept_headers",
             [](HeaderChain& c, const std::vector<BlockHeader>& hs, int64_t adjusted_time, bool check_pow,
                const py::object& hashes, const py::object& bits) {
                 std::vector<Uint256> known;
                 std::vector<u32> kbits;
                 if (!hashes.is_none()) {  // n x 32 bytes, storage order
                     const std::string b = hashes.cast<py::bytes>();
                     if (b.size() != hs.size() * 32) throw std::invalid_argument("hashes: expected 32 bytes per header");
                     known.resize(hs.size());
                     for (size_t i = 0; i < hs.size(); ++i)
                         known[i] = Uint256::from_bytes(reinterpret_cast<const u8*>(b.data()) + 32 * i);
                 }
                 if (!bits.is_none()) {  // n little-endian u32
                     const std::string b = bits.cast<py::bytes>();
                     if (b.size() != hs.size() * 4) throw std::invalid_argument("bits: expected 4 bytes per header");
                     kbits.resize(hs.size());
                     std::memcpy(kbits.data(), b.data(), b.size());
                 }
                 py::gil_scoped_release rel;
                 return c.accept_headers(hs, adjusted_time, check_pow, known.empty() ? nullptr : &known,
                                         kbits.empty() ? nullptr : &kbits);
             },
             py::arg("headers"), py::arg("adjusted_time"), py::arg("check_pow") = true, py::arg("hashes") = py::none(),
             py::arg("bits") = py::none())
        .def("accept_headers_summary",
             [](HeaderChain& c, const std::vector<BlockHeader>& hs, int64_t adjusted_time, bool check_pow,
                const py::object& hashes, const py::object& bits) {
                 // accept_headers for large batches without one Python object per header:
                 // (accepted, reject reason or None, dos)
                 std::vector<Uint256> known;
                 std::vector<u32> kbits;
                 if (!hashes.is_none()) {
                     const std::string b = hashes.cast<py::bytes>();
                     if (b.size() != hs.size() * 32) throw std::invalid_argument("hashes: expected 32 bytes per header");
                     known.resize(hs.size());
                     for (size_t i = 0; i < hs.size(); ++i)
                         known[i] = Uint256::from_bytes(reinterpret_cast<const u8*>(b.data()) + 32 * i);
                 }
                 if (!bits.is_none()) {
                     const std::string b = bits.cast<py::bytes>();
                     if (b.size() != hs.size() * 4) throw std::invalid_argument("bits: expected 4 bytes per header");
                     kbits.resize(hs.size());
                     std::memcpy(kbits.data(), b.data(), b.size());
                 }
                 std::vector<AcceptResult> r;
                 {
                     py::gil_scoped_release rel;
                     r = c.accept_headers(hs, adjusted_time, check_pow, known.empty() ? nullptr : &known,
                                          kbits.empty() ? nullptr : &kbits);
                 }
                 size_t ok = 0;
                 while (ok < r.size() && r[ok].ok) ++ok;
                 py::object why = py::none();
                 int dos = 0;
                 if (ok < r.size()) {
                     why = py::str(r[ok].reject);
                     dos = r[ok].dos;
                 }
                 return py::make_tuple(ok, why, dos);
             },
             py::arg("headers"), py::arg("adjusted_time"), py::arg("check_pow") = true, py::arg("hashes") = py::none(),
             py::arg("bits") = py::none())
        .def("dgw_series",
             [](const HeaderChain& c, const std::vector<BlockHeader>& hs, const py::bytes& hashes) -> py::object {
                 const std::string b = hashes;
                 if (b.size() != hs.size() * 32) throw std::invalid_argument("hashes: expected 32 bytes per header");
                 std::vector<Uint256> hv(hs.size());
                 for (size_t i = 0; i < hs.size(); ++i) hv[i] = Uint256::from_bytes(reinterpret_cast<const u8*>(b.data()) + 32 * i);
                 std::vector<u32> times, bits;
                 size_t a = 0;
                 int base = 0;
                 if (!c.dgw_series(hs, hv, times, bits, a, base)) return py::none();
                 return py::make_tuple(py::bytes(reinterpret_cast<const char*>(times.data()), times.size() * 4),
                                       py::bytes(reinterpret_cast<const char*>(bits.data()), bits.size() * 4), a, base);
             },
             "(times, bits, a, base_height) of a linear batch (u32 little-endian series), or None")
        .def("tip", &HeaderChain::tip, py::return_value_policy::reference_internal)
        .def("genesis", &HeaderChain::genesis, py::return_value_policy::reference_internal)
        .def("at_height", &HeaderChain::at_height, py::return_value_policy::reference_internal)
        .def("find", [](const HeaderChain& c, const py::bytes& h) { return c.find(u256(h)); }, py::return_value_policy::reference_internal)
        .def("in_active_chain", &HeaderChain::in_active_chain)
        .def("height", &HeaderChain::height)
        .def("size", &HeaderChain::size)
        .def("next_bits", &HeaderChain::next_bits)
        .def("invalidate", [](HeaderChain& c, const py::bytes& h) { c.invalidate(u256(h)); })
        .def("reconsider", [](HeaderChain& c, const py::bytes& h) { c.reconsider(u256(h)); })
        .def("block_hash", [](const HeaderChain& c, const BlockHeader& h) { return pyb(c.verifier().block_hash(h, c.params())); })
        .def("block_hash_full", [](const HeaderChain& c, const BlockHeader& h) {
            Uint256 mix;
            Uint256 pow;
            {
                py::gil_scoped_release rel;
                pow = c.verifier().block_hash_full(h, c.params(), mix);
            }
            return py::make_tuple(pyb(pow), pyb(mix));
        })
        .def("dgw", [](const HeaderChain& c, const BlockHeader& next) { return dark_gravity_wave(c.tip(), next, c.params()); });

    py::class_<BlockStore::Pos>(m, "BlockPos")
        .def(py::init<>())
        .def_readwrite("file", &BlockStore::Pos::file)
        .def_readwrite("offset", &BlockStore::Pos::offset)
        .def_readwrite("size", &BlockStore::Pos::size)
        .def(py::pickle([](const BlockStore::Pos& p) { return py::make_tuple(p.file, p.offset, p.size); },
                        [](py::tuple t) { BlockStore::Pos p; p.file = t[0].cast<int>(); p.offset = t[1].cast<u32>(); p.size = t[2].cast<u32>(); return p; }));
    py::class_<BlockStore, std::shared_ptr<BlockStore>>(m, "BlockStore")
        .def(py::init([](const std::string& dir, const py::bytes& magic, u32 act) {
            std::string mg = magic;
            if (mg.size() != 4) throw std::invalid_argument("magic must be 4 bytes");
            return std::make_shared<BlockStore>(dir, reinterpret_cast<const u8*>(mg.data()), act);
        }))
        .def("write", &BlockStore::write)
        .def("write_raw", [](BlockStore& s, const py::bytes& b) { return s.write_raw(bytes_of(b)); })
        .def("read_raw", [](const BlockStore& s, const BlockStore::Pos& p) { return pyb(s.read_raw(p)); })
        .def("read", &BlockStore::read)
        .def("scan", [](const BlockStore& s) { py::list l; for (auto& kv : s.scan()) l.append(py::make_tuple(kv.first, pyb(kv.second))); return l; })
        .def("path", &BlockStore::path)
        .def("current_file", &BlockStore::current_file)
        .def("set_max_file_size", &BlockStore::set_max_file_size);

    // ------------------------------------------------ block validation
    auto bc = [](const BlockCheck& c) { return py::make_tuple(c.ok, c.reject, c.dos); };
    m.def("check_block", [bc](const Block& b, const ChainParams& p, bool merkle, const assets::Flags& f) {
        return bc(check_block(b, p, merkle, f));
    }, py::arg("block"), py::arg("params"), py::arg("check_merkle") = true, py::arg("asset_flags") = assets::Flags{});
    m.def("contextual_check_block", [bc](const Block& b, const ChainParams& p, int h) { return bc(contextual_check_block(b, p, h)); });
    m.def("check_coinbase_rewards", [bc](const Block& b, const ChainParams& p, int h, Amount fees, bool known) {
        return bc(check_coinbase_rewards(b, p, h, fees, known));
    });
    m.def("coinbase_height_prefix", [](int h) { return pyb(coinbase_height_prefix(h)); });

    // ------------------------------------------------ Equihash (CPU reference)
    bind_equihash_cpu(m);
}
