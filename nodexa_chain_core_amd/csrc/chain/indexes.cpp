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

ChainIndexes::Key ChainIndexes::key(int type, const u8 h160[20], const std::string& asset) {
    Key k(1, char(type));
    k.append(reinterpret_cast<const char*>(h160), 20);
    k += asset;
    return k;
}

void ChainIndexes::connect(const Block& block, int height, const Uint256& hash, const BlockUndo& undo) {
    if (timestampindex) time_.emplace(block.header.time, hash);
    for (size_t t = 0; t < block.vtx.size(); ++t) {
        const Transaction& tx = block.vtx[t];
        const Uint256 txid = tx.txid();
        if (txindex) tx_[txid] = hash;
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
                    auto it = unspent_.find(k);
                    if (it != unspent_.end()) {
                        it->second.erase({tx.vin[i].prevout.hash, tx.vin[i].prevout.n});
                        if (it->second.empty()) unspent_.erase(it);
                    }
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
                if (!assets::script_unspendable(tx.vout[n].script_pubkey))
                    unspent_[k][{txid, n}] = {txid, n, amount, tx.vout[n].script_pubkey, height};
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
    }
    for (size_t t = block.vtx.size(); t-- > 0;) {
        const Transaction& tx = block.vtx[t];
        const Uint256 txid = tx.txid();
        if (txindex) {
            auto it = tx_.find(txid);
            if (it != tx_.end() && it->second == hash) tx_.erase(it);
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
                    unspent_[k][{tx.vin[i].prevout.hash, tx.vin[i].prevout.n}] = {
                        tx.vin[i].prevout.hash, tx.vin[i].prevout.n, amount, c.out.script_pubkey, int(c.height)};
                }
                if (spentindex) spent_.erase({tx.vin[i].prevout.hash, tx.vin[i].prevout.n});
            }
        }
    }
    for (auto& k : touched) {  // this block's deltas are the newest entries of each touched address
        auto it = deltas_.find(k);
        if (it == deltas_.end()) continue;
        auto& v = it->second;
        while (!v.empty() && v.back().height >= height) v.pop_back();
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

}  // namespace nodexa
