// Optional chain indexes: see indexes.hpp.
#include "indexes.hpp"

#include <algorithm>

#include "assets.hpp"
#include "script.hpp"
#include "serialize.hpp"

namespace nodexa {

bool index_address(const Bytes& s, int& type, u8 h160[20], std::string& asset, int64_t& amount, int64_t value) {
    asset = "CLORE";
    amount = value;
    if (s.size() == 23 && s[0] == OP_HASH160 && s[1] == 20 && s[22] == OP_EQUAL) {
        type = 2;
        std::memcpy(h160, s.data() + 2, 20);
        return true;
    }
    if (s.size() == 25 && s[0] == OP_DUP && s[1] == OP_HASH160 && s[2] == 20 && s[23] == OP_EQUALVERIFY &&
        s[24] == OP_CHECKSIG) {
        type = 1;
        std::memcpy(h160, s.data() + 3, 20);
        return true;
    }
    if ((s.size() == 35 && s[0] == 33 && s[34] == OP_CHECKSIG) || (s.size() == 67 && s[0] == 65 && s[66] == OP_CHECKSIG)) {
        type = 1;
        hash160(s.data() + 1, s.size() - 2, h160);
        return true;
    }
    assets::AssetOut a;
    if (assets::parse_asset_out(s, a)) {
        type = 1;
        std::memcpy(h160, a.h160, 20);
        asset = a.name;
        amount = a.amount;
        return true;
    }
    return false;
}

namespace {

// record encodings of the reference's index keys/values (addressindex.h, spentindex.h,
// timestampindex.h, txdb.h CDiskTxPos): big-endian heights / positions in keys so that they sort
void put_be32(std::string& s, u32 v) {
    for (int i = 3; i >= 0; --i) s.push_back(char(v >> (8 * i)));
}
void put_le32(std::string& s, u32 v) {
    for (int i = 0; i < 4; ++i) s.push_back(char(v >> (8 * i)));
}
void put_le64(std::string& s, u64 v) {
    for (int i = 0; i < 8; ++i) s.push_back(char(v >> (8 * i)));
}
void put_u256(std::string& s, const Uint256& u) { s.append(reinterpret_cast<const char*>(u.data), 32); }
void put_compact(std::string& s, u64 n) {
    Writer w;
    w.compact_size(n);
    s.append(reinterpret_cast<const char*>(w.buf.data()), w.buf.size());
}
// 'a' / 'u' key prefix: type, hash160, asset name (serialized std::string)
std::string addr_prefix(char p, const std::string& k) {
    std::string s(1, p);
    s.append(k, 0, 21);
    put_compact(s, k.size() - 21);
    s.append(k, 21, std::string::npos);
    return s;
}
std::string delta_key(const std::string& k, const AddrDelta& d) {
    std::string s = addr_prefix('a', k);
    put_be32(s, u32(d.height));
    put_be32(s, d.tx_index);
    put_u256(s, d.txid);
    put_le32(s, d.index);
    s.push_back(d.spending ? 1 : 0);
    return s;
}
std::string le64_str(int64_t v) {
    std::string s;
    put_le64(s, u64(v));
    return s;
}
std::string unspent_key(const std::string& k, const Uint256& txid, u32 n) {
    std::string s = addr_prefix('u', k);
    put_u256(s, txid);
    put_le32(s, n);
    return s;
}
std::string unspent_value(const AddrUnspent& u) {
    std::string s;
    put_le64(s, u64(u.amount));
    put_compact(s, u.script.size());
    s.append(reinterpret_cast<const char*>(u.script.data()), u.script.size());
    put_le32(s, u32(u.height));
    return s;
}
std::string spent_key(const Uint256& txid, u32 n) {
    std::string s(1, 'p');
    put_u256(s, txid);
    put_le32(s, n);
    return s;
}
std::string spent_value(const SpentInfo& si) {
    std::string s;
    put_u256(s, si.txid);
    put_le32(s, si.input);
    put_le32(s, u32(si.height));
    put_le64(s, u64(si.amount));
    put_le32(s, u32(si.addr_type));
    s.append(reinterpret_cast<const char*>(si.h160), 20);
    return s;
}
std::string time_key(u32 t, const Uint256& h) {
    std::string s(1, 's');
    put_be32(s, t);
    put_u256(s, h);
    return s;
}
std::string tx_key(const Uint256& txid) {
    std::string s(1, 't');
    put_u256(s, txid);
    return s;
}

}  // namespace

ChainIndexes::Key ChainIndexes::key(int type, const u8 h160[20], const std::string& asset) {
    Key k(1, char(type));
    k.append(reinterpret_cast<const char*>(h160), 20);
    k += asset;
    return k;
}

void ChainIndexes::connect(const Block& block, int height, const Uint256& hash, const BlockUndo& undo, int file,
                           u32 data_pos) {
    if (timestampindex) {
        time_.emplace(block.header.time, hash);
        rec_put(time_key(block.header.time, hash), std::string(4, '\0'));
        std::string z(1, 'z'), ts;
        put_u256(z, hash);
        put_be32(ts, block.header.time);
        rec_put(z, ts);
    }
    // CDiskTxPos offsets count from the end of the header: CompactSize(#tx), then each tx in turn
    u64 tx_off = 0;
    if (txindex && journal && file >= 0) {
        Writer w;
        w.compact_size(block.vtx.size());
        tx_off = w.buf.size();
    }
    for (size_t t = 0; t < block.vtx.size(); ++t) {
        const Transaction& tx = block.vtx[t];
        const Uint256 txid = tx.txid();
        if (txindex) {
            tx_[txid] = hash;
            if (journal && file >= 0) {
                Bytes pos;
                append_varint(pos, u64(file));
                append_varint(pos, data_pos);
                append_varint(pos, tx_off);
                rec_put(tx_key(txid), std::string(pos.begin(), pos.end()));
                tx_off += tx.bytes(true).size();
            }
        }
        if ((addressindex || spentindex) && !tx.is_coinbase() && t - 1 < undo.vtxundo.size()) {
            const TxUndo& tu = undo.vtxundo[t - 1];
            for (size_t i = 0; i < tx.vin.size() && i < tu.prev.size(); ++i) {
                const Coin& c = tu.prev[i];
                int type = 0;
                u8 h[20] = {0};
                std::string asset;
                int64_t amount = 0;
                const bool has = index_address(c.out.script_pubkey, type, h, asset, amount, c.out.value);
                if (addressindex && has) {
                    const Key k = key(type, h, asset);
                    deltas_[k].push_back({height, u32(t), txid, u32(i), true, -amount});
                    rec_put(delta_key(k, deltas_[k].back()), le64_str(-amount));
                    auto it = unspent_.find(k);
                    if (it != unspent_.end()) {
                        it->second.erase({tx.vin[i].prevout.hash, tx.vin[i].prevout.n});
                        if (it->second.empty()) unspent_.erase(it);
                    }
                    rec_erase(unspent_key(k, tx.vin[i].prevout.hash, tx.vin[i].prevout.n));
                }
                if (spentindex) {
                    SpentInfo si;
                    si.txid = txid;
                    si.input = u32(i);
                    si.height = height;
                    si.amount = c.out.value;
                    si.addr_type = has ? type : 0;
                    std::memcpy(si.h160, h, 20);
                    spent_[{tx.vin[i].prevout.hash, tx.vin[i].prevout.n}] = si;
                    rec_put(spent_key(tx.vin[i].prevout.hash, tx.vin[i].prevout.n), spent_value(si));
                }
            }
        }
        if (addressindex) {
            for (u32 n = 0; n < tx.vout.size(); ++n) {
                int type = 0;
                u8 h[20];
                std::string asset;
                int64_t amount = 0;
                if (!index_address(tx.vout[n].script_pubkey, type, h, asset, amount, tx.vout[n].value)) continue;
                const Key k = key(type, h, asset);
                deltas_[k].push_back({height, u32(t), txid, n, false, amount});
                rec_put(delta_key(k, deltas_[k].back()), le64_str(amount));
                if (!assets::script_unspendable(tx.vout[n].script_pubkey)) {
                    const AddrUnspent u{txid, n, amount, tx.vout[n].script_pubkey, height};
                    unspent_[k][{txid, n}] = u;
                    rec_put(unspent_key(k, txid, n), unspent_value(u));
                }
            }
        }
    }
    best_block = hash;
}

void ChainIndexes::disconnect(const Block& block, int height, const Uint256& hash, const BlockUndo& undo) {
    std::set<Key> touched;
    if (timestampindex) {
        auto range = time_.equal_range(block.header.time);
        for (auto it = range.first; it != range.second; ++it)
            if (it->second == hash) {
                time_.erase(it);
                break;
            }
        rec_erase(time_key(block.header.time, hash));
        std::string z(1, 'z');
        put_u256(z, hash);
        rec_erase(z);
    }
    for (size_t t = block.vtx.size(); t-- > 0;) {
        const Transaction& tx = block.vtx[t];
        const Uint256 txid = tx.txid();
        if (txindex) {
            auto it = tx_.find(txid);
            if (it != tx_.end() && it->second == hash) {
                tx_.erase(it);
                rec_erase(tx_key(txid));
            }
        }
        if (addressindex) {
            for (u32 n = 0; n < tx.vout.size(); ++n) {
                int type = 0;
                u8 h[20];
                std::string asset;
                int64_t amount = 0;
                if (!index_address(tx.vout[n].script_pubkey, type, h, asset, amount, tx.vout[n].value)) continue;
                const Key k = key(type, h, asset);
                touched.insert(k);
                auto it = unspent_.find(k);
                if (it != unspent_.end()) {
                    it->second.erase({txid, n});
                    if (it->second.empty()) unspent_.erase(it);
                }
                rec_erase(unspent_key(k, txid, n));
            }
        }
        if ((addressindex || spentindex) && !tx.is_coinbase() && t - 1 < undo.vtxundo.size()) {
            const TxUndo& tu = undo.vtxundo[t - 1];
            for (size_t i = 0; i < tx.vin.size() && i < tu.prev.size(); ++i) {
                const Coin& c = tu.prev[i];
                int type = 0;
                u8 h[20];
                std::string asset;
                int64_t amount = 0;
                if (addressindex && index_address(c.out.script_pubkey, type, h, asset, amount, c.out.value)) {
                    const Key k = key(type, h, asset);
                    touched.insert(k);
                    const AddrUnspent u{tx.vin[i].prevout.hash, tx.vin[i].prevout.n, amount, c.out.script_pubkey,
                                        int(c.height)};
                    unspent_[k][{u.txid, u.index}] = u;
                    rec_put(unspent_key(k, u.txid, u.index), unspent_value(u));
                }
                if (spentindex) {
                    spent_.erase({tx.vin[i].prevout.hash, tx.vin[i].prevout.n});
                    rec_erase(spent_key(tx.vin[i].prevout.hash, tx.vin[i].prevout.n));
                }
            }
        }
    }
    for (auto& k : touched) {  // this block's deltas are the newest entries of each touched address
        auto it = deltas_.find(k);
        if (it == deltas_.end()) continue;
        auto& v = it->second;
        while (!v.empty() && v.back().height >= height) {
            rec_erase(delta_key(k, v.back()));
            v.pop_back();
        }
        if (v.empty()) deltas_.erase(it);
    }
    best_block = block.header.prev;
}

const Uint256* ChainIndexes::tx_block(const Uint256& txid) const {
    auto it = tx_.find(txid);
    return it == tx_.end() ? nullptr : &it->second;
}

std::vector<std::pair<std::string, AddrDelta>> ChainIndexes::deltas(int type, const u8 h160[20],
                                                                    const std::string& asset, int start, int end) const {
    std::vector<std::pair<std::string, AddrDelta>> out;
    const Key prefix = key(type, h160, "");
    for (auto it = deltas_.lower_bound(prefix); it != deltas_.end() && it->first.compare(0, 21, prefix) == 0; ++it) {
        const std::string name = it->first.substr(21);
        if (asset != "*" && name != asset) continue;
        for (auto& d : it->second)
            if ((start == 0 && end == 0) || (d.height >= start && d.height <= end)) out.emplace_back(name, d);
    }
    std::stable_sort(out.begin(), out.end(), [](auto& a, auto& b) {
        if (a.second.height != b.second.height) return a.second.height < b.second.height;
        return a.second.tx_index < b.second.tx_index;
    });
    return out;
}

std::vector<std::pair<std::string, AddrUnspent>> ChainIndexes::unspent(int type, const u8 h160[20],
                                                                       const std::string& asset) const {
    std::vector<std::pair<std::string, AddrUnspent>> out;
    const Key prefix = key(type, h160, "");
    for (auto it = unspent_.lower_bound(prefix); it != unspent_.end() && it->first.compare(0, 21, prefix) == 0; ++it) {
        const std::string name = it->first.substr(21);
        if (asset != "*" && name != asset) continue;
        for (auto& kv : it->second) out.emplace_back(name, kv.second);
    }
    std::stable_sort(out.begin(), out.end(), [](auto& a, auto& b) { return a.second.height < b.second.height; });
    return out;
}

const SpentInfo* ChainIndexes::spent(const Uint256& txid, u32 n) const {
    auto it = spent_.find({txid, n});
    return it == spent_.end() ? nullptr : &it->second;
}

std::vector<Uint256> ChainIndexes::timestamps(u32 low, u32 high) const {
    std::vector<Uint256> out;
    for (auto it = time_.lower_bound(low); it != time_.end() && it->first < high; ++it) out.push_back(it->second);
    return out;
}

// ------------------------------------------------------------------ snapshot
namespace {
void wstr(Writer& w, const std::string& s) { w.var_bytes(Bytes(s.begin(), s.end())); }
std::string rstr(Reader& r) {
    const Bytes b = r.var_bytes();
    return std::string(b.begin(), b.end());
}
}  // namespace

Bytes ChainIndexes::serialize() const {
    Writer w;
    w.u256(best_block);
    w.u8_(u8((txindex ? 1 : 0) | (addressindex ? 2 : 0) | (spentindex ? 4 : 0) | (timestampindex ? 8 : 0)));
    w.compact_size(tx_.size());
    for (auto& [t, b] : tx_) {
        w.u256(t);
        w.u256(b);
    }
    w.compact_size(deltas_.size());
    for (auto& [k, v] : deltas_) {
        wstr(w, k);
        w.compact_size(v.size());
        for (auto& d : v) {
            w.i32_(d.height);
            w.u32_(d.tx_index);
            w.u256(d.txid);
            w.u32_(d.index);
            w.u8_(d.spending ? 1 : 0);
            w.i64_(d.amount);
        }
    }
    w.compact_size(unspent_.size());
    for (auto& [k, m] : unspent_) {
        wstr(w, k);
        w.compact_size(m.size());
        for (auto& [o, u] : m) {
            w.u256(u.txid);
            w.u32_(u.index);
            w.i64_(u.amount);
            w.var_bytes(u.script);
            w.i32_(u.height);
        }
    }
    w.compact_size(spent_.size());
    for (auto& [o, s] : spent_) {
        w.u256(o.first);
        w.u32_(o.second);
        w.u256(s.txid);
        w.u32_(s.input);
        w.i32_(s.height);
        w.i64_(s.amount);
        w.u8_(u8(s.addr_type));
        w.raw(s.h160, 20);
    }
    w.compact_size(time_.size());
    for (auto& [t, h] : time_) {
        w.u32_(t);
        w.u256(h);
    }
    return w.buf;
}

bool ChainIndexes::deserialize(const Bytes& b) {
    ChainIndexes x;
    try {
        Reader r(b);
        x.best_block = r.u256();
        const u8 f = r.u8_();
        x.txindex = f & 1;
        x.addressindex = f & 2;
        x.spentindex = f & 4;
        x.timestampindex = f & 8;
        for (u64 n = r.compact_size(); n--;) {
            const Uint256 t = r.u256();
            x.tx_[t] = r.u256();
        }
        for (u64 n = r.compact_size(); n--;) {
            const Key k = rstr(r);
            auto& v = x.deltas_[k];
            v.resize(size_t(r.compact_size()));
            for (auto& d : v) {
                d.height = r.i32_();
                d.tx_index = r.u32_();
                d.txid = r.u256();
                d.index = r.u32_();
                d.spending = r.u8_() != 0;
                d.amount = r.i64_();
            }
        }
        for (u64 n = r.compact_size(); n--;) {
            const Key k = rstr(r);
            auto& m = x.unspent_[k];
            for (u64 j = r.compact_size(); j--;) {
                AddrUnspent u;
                u.txid = r.u256();
                u.index = r.u32_();
                u.amount = r.i64_();
                u.script = r.var_bytes();
                u.height = r.i32_();
                m[{u.txid, u.index}] = u;
            }
        }
        for (u64 n = r.compact_size(); n--;) {
            std::pair<Uint256, u32> o;
            o.first = r.u256();
            o.second = r.u32_();
            SpentInfo s;
            s.txid = r.u256();
            s.input = r.u32_();
            s.height = r.i32_();
            s.amount = r.i64_();
            s.addr_type = r.u8_();
            std::memcpy(s.h160, r.take(20), 20);
            x.spent_[o] = s;
        }
        for (u64 n = r.compact_size(); n--;) {
            const u32 t = r.u32_();
            x.time_.emplace(t, r.u256());
        }
        if (!r.empty()) return false;
    } catch (const std::exception&) {
        return false;
    }
    *this = std::move(x);
    return true;
}

bool ChainIndexes::load_records(
    const std::function<void(const std::function<void(const std::string&, const std::string&)>&)>& scan,
    const std::function<bool(int, u32, Uint256*)>& tx_block_at) {
    bool ok = true;
    auto be32 = [](const u8* p) { return (u32(p[0]) << 24) | (u32(p[1]) << 16) | (u32(p[2]) << 8) | u32(p[3]); };
    // key after the prefix byte: type, hash160, CompactSize asset length, asset -> (Key, rest offset)
    auto addr = [&](const std::string& k, Key* out, size_t* rest) {
        if (k.size() < 23) return false;
        try {
            Reader r(reinterpret_cast<const u8*>(k.data()) + 22, k.size() - 22);
            const u64 n = r.compact_size();
            const size_t off = 22 + r.pos();
            if (k.size() < off + n) return false;
            *out = k.substr(1, 21) + k.substr(off, size_t(n));
            *rest = off + size_t(n);
            return true;
        } catch (const std::exception&) {
            return false;
        }
    };
    tx_.clear();
    deltas_.clear();
    unspent_.clear();
    spent_.clear();
    time_.clear();
    scan([&](const std::string& k, const std::string& v) {
        const u8* kp = reinterpret_cast<const u8*>(k.data());
        const u8* vp = reinterpret_cast<const u8*>(v.data());
        try {
            switch (k[0]) {
                case 't': {
                    if (!txindex || k.size() != 33) return;
                    const u8* p = vp;
                    u64 file, pos, off;
                    if (!parse_varint(p, vp + v.size(), file) || !parse_varint(p, vp + v.size(), pos) ||
                        !parse_varint(p, vp + v.size(), off)) {
                        ok = false;
                        return;
                    }
                    Uint256 h;
                    if (tx_block_at(int(file), u32(pos), &h)) tx_[Uint256::from_bytes(kp + 1)] = h;
                    return;
                }
                case 'a': {
                    Key key;
                    size_t o;
                    if (!addressindex) return;
                    if (!addr(k, &key, &o) || k.size() != o + 4 + 4 + 32 + 4 + 1 || v.size() != 8) {
                        ok = false;
                        return;
                    }
                    AddrDelta d;
                    d.height = int(be32(kp + o));
                    d.tx_index = be32(kp + o + 4);
                    d.txid = Uint256::from_bytes(kp + o + 8);
                    d.index = load_le32(kp + o + 40);
                    d.spending = kp[o + 44] != 0;
                    d.amount = int64_t(load_le64(vp));
                    deltas_[key].push_back(d);
                    return;
                }
                case 'u': {
                    Key key;
                    size_t o;
                    if (!addressindex) return;
                    if (!addr(k, &key, &o) || k.size() != o + 36) {
                        ok = false;
                        return;
                    }
                    Reader r(vp, v.size());
                    AddrUnspent u;
                    u.txid = Uint256::from_bytes(kp + o);
                    u.index = load_le32(kp + o + 32);
                    u.amount = r.i64_();
                    u.script = r.var_bytes();
                    u.height = r.i32_();
                    unspent_[key][{u.txid, u.index}] = std::move(u);
                    return;
                }
                case 'p': {
                    if (!spentindex) return;
                    if (k.size() != 37 || v.size() != 32 + 4 + 4 + 8 + 4 + 20) {
                        ok = false;
                        return;
                    }
                    Reader r(vp, v.size());
                    SpentInfo si;
                    si.txid = r.u256();
                    si.input = r.u32_();
                    si.height = r.i32_();
                    si.amount = r.i64_();
                    si.addr_type = r.i32_();
                    std::memcpy(si.h160, r.take(20), 20);
                    spent_[{Uint256::from_bytes(kp + 1), load_le32(kp + 33)}] = si;
                    return;
                }
                case 's':
                    if (!timestampindex) return;
                    if (k.size() != 37) {
                        ok = false;
                        return;
                    }
                    time_.emplace(be32(kp + 1), Uint256::from_bytes(kp + 5));
                    return;
                default: return;
            }
        } catch (const std::exception&) {
            ok = false;
        }
    });
    // deltas in (height, position) order, as connect appends them
    for (auto& kv : deltas_)
        std::stable_sort(kv.second.begin(), kv.second.end(), [](const AddrDelta& a, const AddrDelta& b) {
            return a.height != b.height ? a.height < b.height : a.tx_index < b.tx_index;
        });
    changes_.clear();
    return ok;
}

}  // namespace nodexa
