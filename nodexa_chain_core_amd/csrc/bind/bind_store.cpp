// Bindings for the LevelDB-format store (store/ldb.hpp).
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../store/bdb.hpp"
#include "../store/chaindb.hpp"
#include "../store/ldb.hpp"

namespace py = pybind11;
using namespace nodexa;

void bind_store(py::module_& m) {
    py::class_<ldb::DB>(m, "LevelDB", "A LevelDB-format store directory (blocks/index, chainstate, ...)")
        .def(py::init([](const std::string& path, bool create_if_missing, size_t write_buffer_size, int bloom_bits,
                         size_t max_file_size, size_t block_size, int l0_trigger, uint64_t level1_bytes,
                         size_t max_open_files) {
                 ldb::Options o;
                 o.create_if_missing = create_if_missing;
                 o.write_buffer_size = write_buffer_size;
                 o.bloom_bits_per_key = bloom_bits;
                 o.max_file_size = max_file_size;
                 o.block_size = block_size;
                 o.l0_compaction_trigger = l0_trigger;
                 o.level1_bytes = level1_bytes;
                 o.max_open_files = max_open_files;
                 return ldb::DB::open(path, o);
             }),
             py::arg("path"), py::arg("create_if_missing") = true, py::arg("write_buffer_size") = size_t(4) << 20,
             py::arg("bloom_bits") = 10, py::arg("max_file_size") = size_t(2) << 20, py::arg("block_size") = 4096,
             py::arg("l0_trigger") = 4, py::arg("level1_bytes") = uint64_t(10) << 20,
             py::arg("max_open_files") = size_t(512))
        .def("get",
             [](ldb::DB& db, const py::bytes& k) -> py::object {
                 std::string v;
                 bool found;
                 {
                     const std::string key = k;
                     py::gil_scoped_release rel;
                     found = db.get(key, &v);
                 }
                 if (!found) return py::none();
                 return py::bytes(v);
             })
        .def("put", [](ldb::DB& db, const py::bytes& k, const py::bytes& v,
                       bool sync) { db.put(std::string(k), std::string(v), sync); },
             py::arg("key"), py::arg("value"), py::arg("sync") = false)
        .def("delete", [](ldb::DB& db, const py::bytes& k, bool sync) { db.del(std::string(k), sync); },
             py::arg("key"), py::arg("sync") = false)
        .def("write",
             [](ldb::DB& db, const py::list& ops, bool sync) {
                 // ops: [(key, value)] puts and [(key, None)] deletes, applied in order as one batch
                 ldb::WriteBatch b;
                 for (const py::handle& h : ops) {
                     py::tuple t = py::reinterpret_borrow<py::tuple>(h);
                     if (t[1].is_none()) b.del(std::string(py::bytes(t[0])));
                     else b.put(std::string(py::bytes(t[0])), std::string(py::bytes(t[1])));
                 }
                 py::gil_scoped_release rel;
                 db.write(b, sync);
             },
             py::arg("ops"), py::arg("sync") = false)
        .def("items",
             [](ldb::DB& db, const py::bytes& start, const py::bytes& end) {
                 std::vector<std::pair<std::string, std::string>> out;
                 {
                     const std::string s = start, e = end;
                     py::gil_scoped_release rel;
                     db.scan(s, e, [&](const std::string& k, const std::string& v) {
                         out.emplace_back(k, v);
                         return true;
                     });
                 }
                 py::list l;
                 for (auto& kv : out) l.append(py::make_tuple(py::bytes(kv.first), py::bytes(kv.second)));
                 return l;
             },
             py::arg("start") = py::bytes(""), py::arg("end") = py::bytes(""),
             "live (key, value) pairs with start <= key < end (empty end: unbounded), in key order")
        .def("compact", &ldb::DB::compact_all, py::call_guard<py::gil_scoped_release>())
        .def("flush", &ldb::DB::flush_memtable, py::call_guard<py::gil_scoped_release>())
        .def("files_per_level", &ldb::DB::files_per_level)
        .def_property_readonly("last_sequence", &ldb::DB::last_sequence)
        .def_property_readonly("disk_bytes", &ldb::DB::disk_bytes)
        .def("close", &ldb::DB::close);
    m.def("ldb_destroy", &ldb::destroy);
    m.def("bdb_read", [](const std::string& path, const std::string& subdb) {
        bdb::Records recs;
        {
            py::gil_scoped_release nogil;
            recs = bdb::read_btree(path, subdb);
        }
        py::list out;
        for (const auto& [k, v] : recs) out.append(py::make_tuple(py::bytes(k), py::bytes(v)));
        return out;
    }, py::arg("path"), py::arg("subdb") = "main",
       "Key/value records of a Berkeley DB btree file's sub-database (read-only; store/bdb.hpp)");
    m.def("bdb_databases", &bdb::databases, "Sub-database names of a Berkeley DB btree file");
    m.def("bdb_write", [](const std::string& path, const py::list& records, const std::string& subdb, uint32_t pagesize) {
        bdb::Records recs;
        for (const auto& r : records) {
            auto t = r.cast<py::tuple>();
            recs.emplace_back(t[0].cast<std::string>(), t[1].cast<std::string>());
        }
        py::gil_scoped_release rel;
        bdb::write_btree(path, std::move(recs), subdb, pagesize);
    }, py::arg("path"), py::arg("records"), py::arg("subdb") = "main", py::arg("pagesize") = 4096,
       "Write (key, value) byte records as a Berkeley DB btree file (sub-database `subdb`; store/bdb.hpp)");
    m.def("ldb_crc32c", [](const py::bytes& b) {
        const std::string s = b;
        return ldb::crc32c(s.data(), s.size());
    });
    m.def("ldb_bloom_hash", [](const py::bytes& b) { return ldb::bloom_hash(std::string(b)); });
    m.def("snappy_uncompress", [](const py::bytes& b) -> py::object {
        const std::string s = b;
        std::string out;
        if (!ldb::snappy_uncompress(s.data(), s.size(), &out)) return py::none();
        return py::bytes(out);
    });

    // ---------------- chain databases (store/chaindb.hpp)
    m.def("chaindb_obfuscation_key",
          [](ldb::DB& db, bool create) { return py::bytes(chaindb::obfuscation_key(db, create)); });
    m.def("chaindb_xor", [](const py::bytes& v, const py::bytes& key) {
        std::string s = v;
        chaindb::xor_obf(s, std::string(key));
        return py::bytes(s);
    });
    m.def("coins_load_ldb", [](CoinsView& view, ldb::DB& db, const py::bytes& obf) {
        chaindb::CoinsLoad r;
        {
            const std::string k = obf;
            py::gil_scoped_release rel;
            r = chaindb::coins_load(view, db, k);
        }
        py::dict d;
        d["have_best"] = r.have_best;
        d["head_blocks"] = r.head_blocks;
        d["coins"] = r.coins;
        d["bad"] = r.bad;
        return d;
    });
    m.def("coins_flush_ldb", [](CoinsView& view, ldb::DB& db, const py::bytes& obf, bool sync, assets::State* st) {
        const std::string k = obf;
        py::gil_scoped_release rel;
        return chaindb::coins_flush(view, db, k, sync, st);
    }, py::arg("view"), py::arg("db"), py::arg("obf"), py::arg("sync"), py::arg("assets") = nullptr);
    m.def("assets_load_ldb", [](assets::State& st, ldb::DB& db, const py::bytes& obf) {
        const std::string k = obf;
        py::gil_scoped_release rel;
        return chaindb::assets_load(st, db, k);
    });
    m.def("assets_import_reference_ldb", [](assets::State& st, ldb::DB& assets_db, ldb::DB* restricted_db) {
        chaindb::RefAssetsLoad r;
        {
            py::gil_scoped_release rel;
            r = chaindb::assets_import_reference(st, assets_db, restricted_db);
        }
        py::dict d;
        d["assets"] = r.metas;
        d["balances"] = r.balances;
        d["tags"] = r.tags;
        d["restrictions"] = r.restrictions;
        d["global_restrictions"] = r.globals;
        d["verifiers"] = r.verifiers;
        d["bad"] = r.bad;
        return d;
    }, py::arg("state"), py::arg("assets_db"), py::arg("restricted_db") = nullptr);
    m.def("coin_db_key", [](const py::bytes& txid, u32 n) {
        const std::string s = txid;
        if (s.size() != 32) throw std::invalid_argument("expected a 32-byte txid");
        OutPoint o;
        o.hash = Uint256::from_bytes(reinterpret_cast<const u8*>(s.data()));
        o.n = n;
        return py::bytes(chaindb::coin_key(o));
    });
    m.def("coin_db_serialize", [](int64_t value, const py::bytes& spk, u32 height, bool coinbase) {
        Coin c;
        c.out.value = value;
        const std::string s = spk;
        c.out.script_pubkey.assign(s.begin(), s.end());
        c.height = height;
        c.coinbase = coinbase;
        const Bytes b = serialize_coin_db(c);
        return py::bytes(reinterpret_cast<const char*>(b.data()), b.size());
    });
    m.def("coin_db_deserialize", [](const py::bytes& v) -> py::object {
        const std::string s = v;
        Coin c;
        if (!deserialize_coin_db(reinterpret_cast<const u8*>(s.data()), s.size(), c)) return py::none();
        return py::make_tuple(c.out.value,
                              py::bytes(reinterpret_cast<const char*>(c.out.script_pubkey.data()), c.out.script_pubkey.size()),
                              c.height, c.coinbase);
    });
    m.def("encode_disk_index",
          [](int height, u32 status, u32 ntx, int file, u32 data_pos, u32 undo_pos, const py::bytes& header, u32 act) {
              chaindb::DiskIndex d;
              d.height = height;
              d.status = status;
              d.ntx = ntx;
              d.file = file;
              d.data_pos = data_pos;
              d.undo_pos = undo_pos;
              const std::string h = header;
              d.header.assign(h.begin(), h.end());
              return py::bytes(chaindb::encode_disk_index(d, act));
          });
    m.def("decode_disk_index", [](const py::bytes& v, u32 act) -> py::object {
        chaindb::DiskIndex d;
        if (!chaindb::decode_disk_index(std::string(v), act, &d)) return py::none();
        return py::make_tuple(d.height, d.status, d.ntx, d.file, d.data_pos, d.undo_pos,
                              py::bytes(reinterpret_cast<const char*>(d.header.data()), d.header.size()));
    });
    m.def("load_block_index_ldb", [](ldb::DB& db, const py::bytes& obf, u32 act) {
        std::vector<chaindb::DiskIndex> v;
        size_t bad = 0;
        {
            const std::string k = obf;
            py::gil_scoped_release rel;
            v = chaindb::load_block_index(db, k, act, &bad);
        }
        py::list out;
        for (const auto& d : v)
            out.append(py::make_tuple(py::bytes(reinterpret_cast<const char*>(d.hash.data), 32), d.height, d.status,
                                      d.ntx, d.file, d.data_pos, d.undo_pos,
                                      py::bytes(reinterpret_cast<const char*>(d.header.data()), d.header.size())));
        return py::make_tuple(out, bad);
    });
    m.def("indexes_flush_ldb", [](ChainIndexes& ix, ldb::DB& db, const py::bytes& obf, bool sync) {
        const std::string k = obf;
        py::gil_scoped_release rel;
        return chaindb::indexes_flush(ix, db, k, sync);
    });
    m.def("indexes_load_ldb", [](ChainIndexes& ix, ldb::DB& db, const py::bytes& obf, const py::dict& block_at) {
        // block_at: {(file, data_pos): block hash}
        std::map<std::pair<int, u32>, Uint256> at;
        for (auto kv : block_at) {
            auto key = kv.first.cast<std::pair<int, u32>>();
            const std::string h = kv.second.cast<py::bytes>();
            if (h.size() == 32) at[key] = Uint256::from_bytes(reinterpret_cast<const u8*>(h.data()));
        }
        bool have_best = false, ok;
        {
            const std::string k = obf;
            py::gil_scoped_release rel;
            ok = chaindb::indexes_load(ix, db, k, [&](int f, u32 p, Uint256* out) {
                auto it = at.find({f, p});
                if (it == at.end()) return false;
                *out = it->second;
                return true;
            }, &have_best);
        }
        return py::make_tuple(ok, have_best);
    });
    m.def("indexes_purge_ldb", [](ldb::DB& db) { chaindb::indexes_purge(db); });
    m.def("encode_file_info",[](u32 blocks, u32 size, u32 undo_size, u32 hfirst, u32 hlast, u64 tfirst, u64 tlast) {
        chaindb::FileInfo f{blocks, size, undo_size, hfirst, hlast, tfirst, tlast};
        return py::bytes(chaindb::encode_file_info(f));
    });
    m.def("decode_file_info", [](const py::bytes& v) -> py::object {
        chaindb::FileInfo f;
        if (!chaindb::decode_file_info(std::string(v), &f)) return py::none();
        return py::make_tuple(f.blocks, f.size, f.undo_size, f.height_first, f.height_last, f.time_first, f.time_last);
    });
}
