// Cross-check harness: the reference's own LevelDB library (compiled from its source tree by
// tools/ref_leveldb.sh into build/, never shipped) driven through its public API, so tests can
// check that directories written by nodexa's store (csrc/store/ldb.cpp) open in the reference
// and the other way round.
//
//   ref_leveldb_tool dump <dir>            every live "hexkey hexvalue" line, iterator order
//   ref_leveldb_tool get <dir>             hex keys on stdin -> "hexvalue" or "-" per line
//   ref_leveldb_tool load <dir> <wbuf>     "P hexkey hexvalue" / "D hexkey" lines on stdin,
//                                          100 ops per write batch, write buffer <wbuf> bytes
//   ref_leveldb_tool compact <dir>         CompactRange over everything
//
// Options match CDBWrapper (src/dbwrapper.cpp:103-110): bloom filter 10 bits/key, no
// compression; reads verify checksums and open with paranoid checks.
#include <cstdio>
#include <iostream>
#include <memory>
#include <string>

#include "leveldb/db.h"
#include "leveldb/filter_policy.h"
#include "leveldb/write_batch.h"

static std::string hex(const leveldb::Slice& s) {
    static const char* d = "0123456789abcdef";
    std::string o;
    for (size_t i = 0; i < s.size(); ++i) {
        o.push_back(d[uint8_t(s[i]) >> 4]);
        o.push_back(d[uint8_t(s[i]) & 15]);
    }
    return o;
}
static std::string unhex(const std::string& h) {
    std::string o;
    for (size_t i = 0; i + 1 < h.size(); i += 2) o.push_back(char(std::stoi(h.substr(i, 2), nullptr, 16)));
    return o;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const std::string cmd = argv[1], dir = argv[2];
    leveldb::Options opt;
    opt.filter_policy = leveldb::NewBloomFilterPolicy(10);
    opt.compression = leveldb::kNoCompression;
    opt.paranoid_checks = true;
    opt.create_if_missing = cmd == "load";
    if (cmd == "load" && argc > 3) opt.write_buffer_size = size_t(std::stoull(argv[3]));
    leveldb::DB* raw = nullptr;
    leveldb::Status st = leveldb::DB::Open(opt, dir, &raw);
    if (!st.ok()) {
        std::cerr << "open: " << st.ToString() << "\n";
        return 1;
    }
    std::unique_ptr<leveldb::DB> db(raw);
    leveldb::ReadOptions ro;
    ro.verify_checksums = true;
    if (cmd == "dump") {
        std::unique_ptr<leveldb::Iterator> it(db->NewIterator(ro));
        for (it->SeekToFirst(); it->Valid(); it->Next()) std::cout << hex(it->key()) << " " << hex(it->value()) << "\n";
        if (!it->status().ok()) {
            std::cerr << "iterate: " << it->status().ToString() << "\n";
            return 1;
        }
    } else if (cmd == "get") {
        std::string k;
        while (std::cin >> k) {
            std::string v;
            leveldb::Status s = db->Get(ro, unhex(k), &v);
            if (s.ok()) std::cout << hex(v) << "\n";
            else if (s.IsNotFound()) std::cout << "-\n";
            else {
                std::cerr << "get: " << s.ToString() << "\n";
                return 1;
            }
        }
    } else if (cmd == "load") {
        leveldb::WriteBatch b;
        int n = 0;
        std::string op, k, v;
        while (std::cin >> op >> k) {
            if (op == "P") {
                std::cin >> v;
                if (v == "_") v.clear();
                b.Put(unhex(k), unhex(v));
            } else {
                b.Delete(unhex(k));
            }
            if (++n % 100 == 0) {
                st = db->Write(leveldb::WriteOptions(), &b);
                if (!st.ok()) return 1;
                b.Clear();
            }
        }
        st = db->Write(leveldb::WriteOptions(), &b);
        if (!st.ok()) return 1;
    } else if (cmd == "compact") {
        db->CompactRange(nullptr, nullptr);
    } else {
        return 2;
    }
    db.reset();
    delete opt.filter_policy;
    return 0;
}
