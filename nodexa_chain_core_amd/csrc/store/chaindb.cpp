// Chain databases in the reference's key layout: see chaindb.hpp.
#include "chaindb.hpp"

#include <algorithm>
#include <cstring>
#include <random>
#include <stdexcept>

#include "../chain/primitives.hpp"
#include "../chain/script.hpp"

namespace nodexa {
namespace chaindb {

namespace {

const std::string kObfKey = std::string("\x0e\x00obfuscate_key", 15);  // CompactSize(14) + "\0obfuscate_key"

std::string bytes_str(const Bytes& b) { return std::string(reinterpret_cast<const char*>(b.data()), b.size()); }

}  // namespace

std::string obfuscation_key(ldb::DB& db, bool create) {
    std::string v;
    if (db.get(kObfKey, &v)) {
        // a serialized vector<unsigned char>: CompactSize(8) + 8 bytes (written before any key
        // was in force, so not itself obfuscated)
        if (v.size() == 9 && uint8_t(v[0]) == 8) return v.substr(1);
        throw std::runtime_error("chaindb: malformed obfuscation key record");
    }
    bool empty = true;
    db.scan(std::string(), std::string(), [&](const std::string&, const std::string&) {
        empty = false;
        return false;
    });
    if (!create || !empty) return std::string(8, '\0');
    std::random_device rd;
    std::string key(8, '\0');
    for (char& c : key) c = char(rd() & 0xff);
    db.put(kObfKey, std::string(1, '\x08') + key, true);
    return key;
}

void xor_obf(std::string& v, const std::string& key) {
    if (key.empty()) return;
    const size_t k = key.size();
    for (size_t i = 0; i < v.size(); ++i) v[i] ^= key[i % k];
}

std::string coin_key(const OutPoint& o) {
    Bytes k;
    k.reserve(40);
    k.push_back('C');
    k.insert(k.end(), o.hash.data, o.hash.data + 32);
    append_varint(k, o.n);
    return bytes_str(k);
}

CoinsLoad coins_load(CoinsView& view, ldb::DB& db, const std::string& obf) {
    CoinsLoad r;
    view.reset();
    std::string v;
    if (db.get("B", &v)) {
        xor_obf(v, obf);
        if (v.size() == 32) {
            view.best_block = Uint256::from_bytes(reinterpret_cast<const u8*>(v.data()));
            r.have_best = true;
        }
    }
    r.head_blocks = db.get("H", &v);
    db.scan("C", "D", [&](const std::string& k, const std::string& val) {
        const u8* p = reinterpret_cast<const u8*>(k.data()) + 1;
        const u8* end = reinterpret_cast<const u8*>(k.data()) + k.size();
        u64 n;
        if (k.size() < 34) {
            ++r.bad;
            return true;
        }
        OutPoint o;
        o.hash = Uint256::from_bytes(p);
        p += 32;
        if (!parse_varint(p, end, n) || p != end || n > 0xffffffffu) {
            ++r.bad;
            return true;
        }
        o.n = u32(n);
        std::string dv = val;
        xor_obf(dv, obf);
        Coin c;
        if (!deserialize_coin_db(reinterpret_cast<const u8*>(dv.data()), dv.size(), c)) {
            ++r.bad;
            return true;
        }
        view.insert_clean(o, std::move(c));
        ++r.coins;
        return true;
    });
    view.clear_dirty();
    return r;
}

namespace {
const std::string kAssetsBest = "\x02" "assets.best";

void put_str(std::string& s, const std::string& v) {
    Writer w;
    w.compact_size(v.size());
    s.append(reinterpret_cast<const char*>(w.buf.data()), w.buf.size());
    s += v;
}
}  // namespace

bool assets_load(assets::State& st, ldb::DB& db, const std::string& obf) {
    st.reset();
    std::string v;
    if (!db.get(kAssetsBest, &v)) return false;
    xor_obf(v, obf);
    if (v.size() != 32) return false;
    bool ok = true;
    db.scan("\x01", "\x02", [&](const std::string& k, const std::string& val) {
        try {
            if (k.size() < 2) throw std::runtime_error("short key");
            Reader r(reinterpret_cast<const u8*>(k.data()) + 2, k.size() - 2);
            const Bytes a = r.var_bytes(), bb = r.var_bytes();
            std::string dv = val;
            xor_obf(dv, obf);
            if (!r.empty() || !st.load_entry(u8(k[1]), std::string(a.begin(), a.end()), std::string(bb.begin(), bb.end()),
                                             Bytes(dv.begin(), dv.end())))
                ok = false;
        } catch (const std::exception&) {
            ok = false;
        }
        return ok;
    });
    st.best_block = Uint256::from_bytes(reinterpret_cast<const u8*>(v.data()));
    st.clear_dirty();
    return ok;
}

namespace {
// CDBWrapper keys of the asset databases: a flag char, then one or two serialized strings.
bool ref_key(const std::string& k, char flag, int nstr, std::string& a, std::string& b) {
    if (k.empty() || k[0] != flag) return false;
    try {
        Reader r(reinterpret_cast<const u8*>(k.data()) + 1, k.size() - 1);
        const Bytes x = r.var_bytes();
        a.assign(x.begin(), x.end());
        if (nstr == 2) {
            const Bytes y = r.var_bytes();
            b.assign(y.begin(), y.end());
        }
        return r.empty();
    } catch (const std::exception&) {
        return false;
    }
}

// An address of the reference's records as this engine's 20-byte balance / tag key.
bool ref_addr20(const std::string& addr, std::string& out) {
    Bytes payload;
    if (!base58check_decode(addr, payload) || payload.size() != 21) return false;
    out.assign(reinterpret_cast<const char*>(payload.data()) + 1, 20);
    return true;
}

// ReadWriteAssetHash (src/assets/assettypes.h:59-95): 0x12 + 32 bytes -> "\x12\x20" + 32 bytes,
// any other tag (the txid notifier) -> the 32 bytes.
std::string ref_asset_hash(Reader& r) {
    const u8 tag = r.u8_();
    const Bytes h = r.var_bytes();
    std::string out;
    if (tag == 0x12) out = std::string("\x12\x20", 2);
    out.append(reinterpret_cast<const char*>(h.data()), std::min<size_t>(h.size(), 32));
    return out;
}
}  // namespace

RefAssetsLoad assets_import_reference(assets::State& st, ldb::DB& adb, ldb::DB* rdb) {
    RefAssetsLoad out;
    st.reset();
    auto value = [](ldb::DB& db, std::string v, const std::string& obf) {
        xor_obf(v, obf);
        return v;
    };
    const std::string aobf = obfuscation_key(adb, false);
    // 'A': CDatabasedAssetData = CNewAsset (name, amount, units, reissuable, has_ipfs [, hash]),
    // nHeight, blockHash
    adb.scan("A", "B", [&](const std::string& k, const std::string& v0) {
        std::string name, unused;
        if (!ref_key(k, 'A', 1, name, unused)) {
            ++out.bad;
            return true;
        }
        try {
            const std::string v = value(adb, v0, aobf);
            Reader r(reinterpret_cast<const u8*>(v.data()), v.size());
            assets::Meta m;
            const Bytes n = r.var_bytes();
            m.name.assign(n.begin(), n.end());
            m.amount = r.i64_();
            m.units = int8_t(r.u8_());
            m.reissuable = int8_t(r.u8_());
            m.has_ipfs = int8_t(r.u8_());
            if (m.has_ipfs == 1) m.ipfs = ref_asset_hash(r);
            m.height = r.i32_();
            m.block = r.u256();
            if (m.name != name) throw std::runtime_error("name mismatch");
            st.set_meta(m);
            ++out.metas;
        } catch (const std::exception&) {
            ++out.bad;
        }
        return true;
    });
    // 'B': (asset name, address) -> CAmount
    adb.scan("B", "C", [&](const std::string& k, const std::string& v0) {
        std::string name, addr, key;
        const std::string v = value(adb, v0, aobf);
        if (!ref_key(k, 'B', 2, name, addr) || v.size() != 8 || !ref_addr20(addr, key)) {
            ++out.bad;
            return true;
        }
        int64_t q;
        std::memcpy(&q, v.data(), 8);  // little-endian CAmount
        if (q != 0) st.add_balance(name, reinterpret_cast<const u8*>(key.data()), q);
        ++out.balances;
        return true;
    });
    if (rdb) {
        const std::string robf = obfuscation_key(*rdb, false);
        rdb->scan("G", "H", [&](const std::string& k, const std::string&) {
            std::string name, unused;
            if (!ref_key(k, 'G', 1, name, unused)) ++out.bad;
            else st.set_global(name, true), ++out.globals;
            return true;
        });
        rdb->scan("R", "S", [&](const std::string& k, const std::string&) {
            std::string addr, name, key;
            if (!ref_key(k, 'R', 2, addr, name) || !ref_addr20(addr, key)) ++out.bad;
            else st.set_frozen(name, reinterpret_cast<const u8*>(key.data()), true), ++out.restrictions;
            return true;
        });
        rdb->scan("T", "U", [&](const std::string& k, const std::string&) {
            std::string addr, tag, key;
            if (!ref_key(k, 'T', 2, addr, tag) || !ref_addr20(addr, key)) ++out.bad;
            else st.set_tag(tag, reinterpret_cast<const u8*>(key.data()), true), ++out.tags;
            return true;
        });
        rdb->scan("V", "W", [&](const std::string& k, const std::string& v0) {
            std::string name, unused;
            try {
                const std::string v = value(*rdb, v0, robf);
                Reader r(reinterpret_cast<const u8*>(v.data()), v.size());
                const Bytes ver = r.var_bytes();
                if (!ref_key(k, 'V', 1, name, unused)) throw std::runtime_error("key");
                st.set_verifier(name, std::string(ver.begin(), ver.end()));
                ++out.verifiers;
            } catch (const std::exception&) {
                ++out.bad;
            }
            return true;
        });
    }
    st.clear_journal();  // an imported state has no undo history in this engine
    st.clear_dirty();
    return out;
}

size_t coins_flush(CoinsView& view, ldb::DB& db, const std::string& obf, bool sync, assets::State* assets) {
    ldb::WriteBatch b;
    size_t n = 0;
    if (assets) {
        assets->for_each_dirty([&](u8 kind, const std::string& a, const std::string& k, const Bytes* val) {
            std::string key(1, '\x01');
            key.push_back(char(kind));
            put_str(key, a);
            put_str(key, k);
            if (val) {
                std::string v(val->begin(), val->end());
                if (v.empty()) v = "\x01";  // set members: a present marker
                xor_obf(v, obf);
                b.put(key, v);
            } else {
                b.del(key);
            }
        });
        std::string best(reinterpret_cast<const char*>(assets->best_block.data), 32);
        xor_obf(best, obf);
        b.put(kAssetsBest, best);
    }
    view.for_each_dirty([&](const OutPoint& o, const Coin* c) {
        if (c) {
            std::string v = bytes_str(serialize_coin_db(*c));
            xor_obf(v, obf);
            b.put(coin_key(o), v);
        } else {
            b.del(coin_key(o));
        }
        ++n;
    });
    std::string best(reinterpret_cast<const char*>(view.best_block.data), 32);
    xor_obf(best, obf);
    b.put("B", best);
    b.del("H");
    db.write(b, sync);
    view.clear_dirty();
    if (assets) assets->clear_dirty();
    return n;
}

std::string encode_disk_index(const DiskIndex& d, u32 act, int client_version) {
    Reader hr(d.header);
    const BlockHeader h = BlockHeader::deserialize(hr, act);
    Bytes out;
    append_varint(out, u64(client_version));
    append_varint(out, u64(d.height));
    append_varint(out, d.status);
    append_varint(out, d.ntx);
    if (d.status & (BLOCK_HAVE_DATA | BLOCK_HAVE_UNDO)) append_varint(out, u64(d.file));
    if (d.status & BLOCK_HAVE_DATA) append_varint(out, d.data_pos);
    if (d.status & BLOCK_HAVE_UNDO) append_varint(out, d.undo_pos);
    Writer w;
    w.i32_(h.version);
    w.u256(h.prev);
    w.u256(h.merkle_root);
    w.u32_(h.time);
    w.u32_(h.bits);
    if (h.is_equihash()) {  // this engine's Equihash extension (not a reference header form)
        w.u32_(h.height);
        w.u256(h.nonce256);
        w.var_bytes(h.solution);
    } else if (h.is_kawpow(act)) {
        w.u64_(h.nonce64);
        w.u256(h.mix_hash);
    } else {
        w.u32_(h.nonce);
    }
    out.insert(out.end(), w.buf.begin(), w.buf.end());
    return bytes_str(out);
}

bool decode_disk_index(const std::string& v, u32 act, DiskIndex* d) {
    const u8* p = reinterpret_cast<const u8*>(v.data());
    const u8* end = p + v.size();
    u64 ver, height, status, ntx, file = 0, dpos = 0, upos = 0;
    if (!parse_varint(p, end, ver) || !parse_varint(p, end, height) || !parse_varint(p, end, status) ||
        !parse_varint(p, end, ntx))
        return false;
    if ((status & (BLOCK_HAVE_DATA | BLOCK_HAVE_UNDO)) && !parse_varint(p, end, file)) return false;
    if ((status & BLOCK_HAVE_DATA) && !parse_varint(p, end, dpos)) return false;
    if ((status & BLOCK_HAVE_UNDO) && !parse_varint(p, end, upos)) return false;
    try {
        Reader r(p, size_t(end - p));
        BlockHeader h;
        h.version = r.i32_();
        h.prev = r.u256();
        h.merkle_root = r.u256();
        h.time = r.u32_();
        h.bits = r.u32_();
        if (h.is_equihash()) {
            h.height = r.u32_();
            h.nonce256 = r.u256();
            h.solution = r.var_bytes();
        } else if (h.is_kawpow(act)) {
            h.height = u32(height);
            h.nonce64 = r.u64_();
            h.mix_hash = r.u256();
        } else {
            h.nonce = r.u32_();
        }
        Writer w;
        h.serialize(w, act);
        d->header = std::move(w.buf);
    } catch (const std::exception&) {
        return false;
    }
    d->height = int(height);
    d->status = u32(status);
    d->ntx = u32(ntx);
    d->file = (status & (BLOCK_HAVE_DATA | BLOCK_HAVE_UNDO)) ? int(file) : -1;
    d->data_pos = u32(dpos);
    d->undo_pos = u32(upos);
    return true;
}

std::vector<DiskIndex> load_block_index(ldb::DB& db, const std::string& obf, u32 act, size_t* bad) {
    std::vector<DiskIndex> out;
    size_t nbad = 0;
    db.scan("b", "c", [&](const std::string& k, const std::string& val) {
        if (k.size() != 33) {
            ++nbad;
            return true;
        }
        std::string dv = val;
        xor_obf(dv, obf);
        DiskIndex d;
        if (!decode_disk_index(dv, act, &d)) {
            ++nbad;
            return true;
        }
        d.hash = Uint256::from_bytes(reinterpret_cast<const u8*>(k.data()) + 1);
        out.push_back(std::move(d));
        return true;
    });
    if (bad) *bad = nbad;
    return out;
}

namespace {
const std::string kIndexBest = std::string("\x00nodexa.indexes.best", 20);
const char kIndexPrefixes[] = {'t', 'a', 'u', 'p', 's', 'z'};
}  // namespace

size_t indexes_flush(ChainIndexes& ix, ldb::DB& db, const std::string& obf, bool sync) {
    ldb::WriteBatch b;
    auto ch = ix.take_changes();
    for (auto& c : ch) {
        if (c.second) {
            std::string v = std::move(*c.second);
            xor_obf(v, obf);
            b.put(c.first, v);
        } else {
            b.del(c.first);
        }
    }
    std::string best(reinterpret_cast<const char*>(ix.best_block.data), 32);
    xor_obf(best, obf);
    b.put(kIndexBest, best);
    db.write(b, sync);
    return ch.size();
}

bool indexes_load(ChainIndexes& ix, ldb::DB& db, const std::string& obf,
                  const std::function<bool(int, u32, Uint256*)>& block_at, bool* have_best) {
    std::string v;
    *have_best = false;
    if (db.get(kIndexBest, &v)) {
        xor_obf(v, obf);
        if (v.size() == 32) {
            ix.best_block = Uint256::from_bytes(reinterpret_cast<const u8*>(v.data()));
            *have_best = true;
        }
    }
    return ix.load_records(
        [&](const std::function<void(const std::string&, const std::string&)>& f) {
            for (char p : kIndexPrefixes)
                db.scan(std::string(1, p), std::string(1, char(p + 1)), [&](const std::string& k, const std::string& val) {
                    std::string dv = val;
                    xor_obf(dv, obf);
                    f(k, dv);
                    return true;
                });
        },
        block_at);
}

void indexes_purge(ldb::DB& db) {
    ldb::WriteBatch b;
    for (char p : kIndexPrefixes)
        db.scan(std::string(1, p), std::string(1, char(p + 1)), [&](const std::string& k, const std::string&) {
            b.del(k);
            return true;
        });
    b.del(kIndexBest);
    db.write(b, true);
}

std::string encode_file_info(const FileInfo& f) {
    Bytes out;
    append_varint(out, f.blocks);
    append_varint(out, f.size);
    append_varint(out, f.undo_size);
    append_varint(out, f.height_first);
    append_varint(out, f.height_last);
    append_varint(out, f.time_first);
    append_varint(out, f.time_last);
    return bytes_str(out);
}

bool decode_file_info(const std::string& v, FileInfo* f) {
    const u8* p = reinterpret_cast<const u8*>(v.data());
    const u8* end = p + v.size();
    u64 x[7];
    for (u64& e : x)
        if (!parse_varint(p, end, e)) return false;
    f->blocks = u32(x[0]);
    f->size = u32(x[1]);
    f->undo_size = u32(x[2]);
    f->height_first = u32(x[3]);
    f->height_last = u32(x[4]);
    f->time_first = x[5];
    f->time_last = x[6];
    return true;
}

}  // namespace chaindb
}  // namespace nodexa
