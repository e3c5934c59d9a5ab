// UTXO set, undo data and block connection: see coins.hpp.
#include "coins.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <memory>
#include <thread>
#include <fstream>
#include <map>
#include <set>

#include "../crypto/secp256k1.hpp"
#include "../crypto/sha256.hpp"

namespace nodexa {

// ------------------------------------------------------------------ CoinsView
const Coin* CoinsView::find(const OutPoint& o) const {
    auto it = map_.find(o);
    return it == map_.end() ? nullptr : &it->second;
}

void CoinsView::add(const OutPoint& o, Coin c) {
    map_[o] = std::move(c);
    dirty_[o] = true;
}

bool CoinsView::spend(const OutPoint& o, Coin* moved) {
    auto it = map_.find(o);
    if (it == map_.end()) return false;
    if (moved) *moved = std::move(it->second);
    map_.erase(it);
    dirty_[o] = false;
    return true;
}

namespace {

constexpr char kCoinsMagic[8] = {'N', 'X', 'C', 'O', 'I', 'N', 'S', '1'};   // snapshot, no journal seq
constexpr char kCoinsMagic2[8] = {'N', 'X', 'C', 'O', 'I', 'N', 'S', '2'};  // snapshot + journal seq
constexpr char kJournalMagic[4] = {'N', 'X', 'C', 'J'};

// write(2) the whole buffer and fsync: a journal record is durable before flush returns
void write_all_fsync(int fd, const u8* p, size_t n, const std::string& what) {
    while (n) {
        const ssize_t k = ::write(fd, p, n);
        if (k < 0) {
            if (errno == EINTR) continue;
            throw std::runtime_error("cannot write " + what);
        }
        p += k;
        n -= size_t(k);
    }
    if (::fsync(fd) != 0) throw std::runtime_error("cannot fsync " + what);
}

void write_coin_entry(Writer& w, const OutPoint& o, const Coin& c) {
    w.u256(o.hash);
    w.u32_(o.n);
    w.u32_((c.height << 1) | (c.coinbase ? 1u : 0u));
    w.i64_(c.out.value);
    w.var_bytes(c.out.script_pubkey);
}

std::vector<std::pair<OutPoint, const Coin*>> sorted_coins(
    const std::unordered_map<OutPoint, Coin, OutPointHasher, OutPointEq>& m) {
    std::vector<std::pair<OutPoint, const Coin*>> v;
    v.reserve(m.size());
    for (auto& kv : m) v.emplace_back(kv.first, &kv.second);
    std::sort(v.begin(), v.end(), [](auto& a, auto& b) {
        const int c = std::memcmp(a.first.hash.data, b.first.hash.data, 32);
        return c != 0 ? c < 0 : a.first.n < b.first.n;
    });
    return v;
}

}  // namespace

void CoinsView::save(const std::string& path) const {
    Writer w;
    w.raw(reinterpret_cast<const u8*>(kCoinsMagic2), 8);
    w.u256(best_block);
    w.u64_(journal_seq);
    w.u64_(map_.size());
    for (auto& kv : map_) write_coin_entry(w, kv.first, kv.second);
    u8 sum[32];
    sha256d(w.buf.data(), w.buf.size(), sum);
    w.raw(sum, 32);
    const std::string tmp = path + ".new";
    const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) throw std::runtime_error("cannot write " + tmp);
    try {
        write_all_fsync(fd, w.buf.data(), w.buf.size(), tmp);
    } catch (...) {
        ::close(fd);
        throw;
    }
    ::close(fd);
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("cannot replace " + path);
}

bool CoinsView::load(const std::string& path) {
    map_.clear();
    best_block = Uint256();
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    Bytes b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (b.size() < 8 + 32 + 8 + 32) return false;
    const bool v2 = std::memcmp(b.data(), kCoinsMagic2, 8) == 0;
    if (!v2 && std::memcmp(b.data(), kCoinsMagic, 8) != 0) return false;
    u8 sum[32];
    sha256d(b.data(), b.size() - 32, sum);
    if (std::memcmp(sum, b.data() + b.size() - 32, 32) != 0) return false;
    dirty_.clear();
    try {
        Reader r(b.data() + 8, b.size() - 8 - 32);
        best_block = r.u256();
        journal_seq = v2 ? r.u64_() : 0;
        const u64 n = r.u64_();
        map_.reserve(n);
        for (u64 i = 0; i < n; ++i) {
            OutPoint o;
            o.hash = r.u256();
            o.n = r.u32_();
            Coin c;
            const u32 code = r.u32_();
            c.height = code >> 1;
            c.coinbase = code & 1;
            c.out.value = r.i64_();
            c.out.script_pubkey = r.var_bytes();
            map_.emplace(o, std::move(c));
        }
    } catch (const std::exception&) {
        map_.clear();
        best_block = Uint256();
        journal_seq = 0;
        return false;
    }
    return true;
}

void CoinsView::append_journal(const std::string& journal) {
    Writer pay;
    pay.u64_(journal_seq + 1);
    pay.u256(best_block);
    pay.u64_(dirty_.size());
    for (auto& [o, present] : dirty_) {
        pay.u256(o.hash);
        pay.u32_(o.n);
        const Coin* c = present ? find(o) : nullptr;
        pay.u8_(c ? 1 : 0);
        if (c) {
            pay.u32_((c->height << 1) | (c->coinbase ? 1u : 0u));
            pay.i64_(c->out.value);
            pay.var_bytes(c->out.script_pubkey);
        }
    }
    Writer rec;
    rec.raw(reinterpret_cast<const u8*>(kJournalMagic), 4);
    rec.u32_(u32(pay.buf.size()));
    rec.raw(pay.buf);
    u8 sum[32];
    sha256d(pay.buf.data(), pay.buf.size(), sum);
    rec.raw(sum, 32);
    const int fd = ::open(journal.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd < 0) throw std::runtime_error("cannot open " + journal);
    try {
        write_all_fsync(fd, rec.buf.data(), rec.buf.size(), journal);
    } catch (...) {
        ::close(fd);
        throw;
    }
    ::close(fd);
    ++journal_seq;
    dirty_.clear();
}

bool CoinsView::load_with_journal(const std::string& snapshot, const std::string& journal) {
    const bool have_snapshot = load(snapshot);
    if (!have_snapshot) {  // no (valid) snapshot: the journal alone is replayed from sequence 1
        map_.clear();
        best_block = Uint256();
        journal_seq = 0;
    }
    replayed = 0;
    std::ifstream f(journal, std::ios::binary);
    if (!f) return have_snapshot;
    Bytes b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    f.close();
    size_t pos = 0, good = 0;
    while (b.size() - pos >= 8 + 32) {
        if (std::memcmp(b.data() + pos, kJournalMagic, 4) != 0) break;
        const u32 len = load_le32(b.data() + pos + 4);
        if (b.size() - pos - 8 < size_t(len) + 32) break;  // torn tail record
        const u8* payload = b.data() + pos + 8;
        u8 sum[32];
        sha256d(payload, len, sum);
        if (std::memcmp(sum, payload + len, 32) != 0) break;
        try {
            Reader r(payload, len);
            const u64 seq = r.u64_();
            const Uint256 best = r.u256();
            const u64 n = r.u64_();
            if (seq > journal_seq + 1) break;  // a gap: records after it cannot apply
            if (seq == journal_seq + 1) {
                for (u64 i = 0; i < n; ++i) {
                    OutPoint o;
                    o.hash = r.u256();
                    o.n = r.u32_();
                    if (r.u8_()) {
                        Coin c;
                        const u32 code = r.u32_();
                        c.height = code >> 1;
                        c.coinbase = code & 1;
                        c.out.value = r.i64_();
                        c.out.script_pubkey = r.var_bytes();
                        map_[o] = std::move(c);
                    } else {
                        map_.erase(o);
                    }
                }
                best_block = best;
                journal_seq = seq;
                ++replayed;
            }
        } catch (const std::exception&) {
            break;
        }
        pos += 8 + size_t(len) + 32;
        good = pos;
    }
    if (good < b.size()) {  // cut a torn or corrupt tail so later appends follow a complete record
        if (::truncate(journal.c_str(), off_t(good)) != 0) throw std::runtime_error("cannot truncate " + journal);
    }
    dirty_.clear();
    return have_snapshot || replayed > 0;
}

void CoinsView::compact(const std::string& snapshot, const std::string& journal) {
    if (!dirty_.empty()) append_journal(journal);
    save(snapshot);  // carries journal_seq: every record up to it is now folded in
    const int fd = ::open(journal.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) throw std::runtime_error("cannot truncate " + journal);
    ::fsync(fd);
    ::close(fd);
}

CoinsView::Stats CoinsView::stats() const {
    // hash_serialized_2 as GetUTXOStats / ApplyStats define it (src/rpc/blockchain.cpp:1076-1130):
    // the best block, then per transaction (coins in 'C' key order) its txid, VARINT(height * 2 +
    // coinbase), per output VARINT(n + 1), the script and VARINT(value), closed by VARINT(0)
    Stats s;
    Writer w;
    w.u256(best_block);
    const Uint256* last = nullptr;
    auto close_tx = [&] {
        if (last) append_varint(w.buf, 0);
    };
    for (auto& [o, c] : sorted_coins(map_)) {
        if (!last || std::memcmp(last->data, o.hash.data, 32) != 0) {
            close_tx();
            ++s.transactions;
            w.u256(o.hash);
            append_varint(w.buf, u64(c->height) * 2 + (c->coinbase ? 1 : 0));
        }
        last = &o.hash;
        ++s.txouts;
        s.total += c->out.value;
        append_varint(w.buf, u64(o.n) + 1);
        w.var_bytes(c->out.script_pubkey);
        append_varint(w.buf, u64(c->out.value));
        s.bogosize += 32 + 4 + 4 + 8 + 2 + c->out.script_pubkey.size();
    }
    close_tx();
    sha256d(w.buf.data(), w.buf.size(), s.hash.data);
    return s;
}

// ------------------------------------------------------------------ undo encoding
namespace {

void write_varint(Writer& w, u64 n) {
    u8 tmp[10];
    int len = 0;
    while (true) {
        tmp[len] = u8((n & 0x7F) | (len ? 0x80 : 0x00));
        if (n <= 0x7F) break;
        n = (n >> 7) - 1;
        ++len;
    }
    do {
        w.u8_(tmp[len]);
    } while (len--);
}

u64 read_varint(Reader& r) {
    u64 n = 0;
    while (true) {
        const u8 ch = r.u8_();
        if (n > (~u64(0) >> 7)) throw std::runtime_error("ReadVarInt(): size too large");
        n = (n << 7) | (ch & 0x7F);
        if (ch & 0x80) {
            if (n == ~u64(0)) throw std::runtime_error("ReadVarInt(): size too large");
            ++n;
        } else {
            return n;
        }
    }
}

constexpr u64 kSpecialScripts = 6;

// CScriptCompressor::Compress: the 21/33-byte special forms, or false
bool compress_script(const Bytes& s, Bytes& out) {
    if (s.size() == 25 && s[0] == 0x76 && s[1] == 0xa9 && s[2] == 20 && s[23] == 0x88 && s[24] == 0xac) {
        out.assign(1, 0x00);
        out.insert(out.end(), s.begin() + 3, s.begin() + 23);
        return true;
    }
    if (s.size() == 23 && s[0] == 0xa9 && s[1] == 20 && s[22] == 0x87) {
        out.assign(1, 0x01);
        out.insert(out.end(), s.begin() + 2, s.begin() + 22);
        return true;
    }
    if (s.size() == 35 && s[0] == 33 && s[34] == 0xac && (s[1] == 0x02 || s[1] == 0x03)) {
        out.assign(s.begin() + 1, s.begin() + 34);
        return true;
    }
    if (s.size() == 67 && s[0] == 65 && s[66] == 0xac && s[1] == 0x04) {
        secp::Ge p;
        if (!secp::pubkey_parse(s.data() + 1, 65, p)) return false;  // IsFullyValid
        out.assign(1, u8(0x04 | (s[65] & 0x01)));
        out.insert(out.end(), s.begin() + 2, s.begin() + 34);
        return true;
    }
    return false;
}

Bytes decompress_script(u64 kind, const Bytes& in) {
    Bytes s;
    switch (kind) {
        case 0:
            s = {0x76, 0xa9, 20};
            s.insert(s.end(), in.begin(), in.end());
            s.push_back(0x88);
            s.push_back(0xac);
            return s;
        case 1:
            s = {0xa9, 20};
            s.insert(s.end(), in.begin(), in.end());
            s.push_back(0x87);
            return s;
        case 2:
        case 3:
            s = {33, u8(kind)};
            s.insert(s.end(), in.begin(), in.end());
            s.push_back(0xac);
            return s;
        default: {  // 4, 5: uncompressed key stored as its x and the parity of y
            u8 c[33];
            c[0] = u8(kind - 2);
            std::memcpy(c + 1, in.data(), 32);
            secp::Ge p;
            if (!secp::pubkey_parse(c, 33, p)) return s;
            u8 full[65];
            secp::pubkey_serialize(p, false, full);
            s.push_back(65);
            s.insert(s.end(), full, full + 65);
            s.push_back(0xac);
            return s;
        }
    }
}

void write_coin_undo(Writer& w, const Coin& c) {
    write_varint(w, u64(c.height) * 2 + (c.coinbase ? 1 : 0));
    if (c.height > 0) w.u8_(0);  // the old undo format's nVersion placeholder
    write_varint(w, compress_amount(u64(c.out.value)));
    Bytes comp;
    if (compress_script(c.out.script_pubkey, comp)) {
        w.raw(comp);
    } else {
        write_varint(w, c.out.script_pubkey.size() + kSpecialScripts);
        w.raw(c.out.script_pubkey);
    }
}

Coin read_coin_undo(Reader& r) {
    Coin c;
    const u64 code = read_varint(r);
    c.height = u32(code >> 1);
    c.coinbase = code & 1;
    if (c.height > 0) (void)read_varint(r);
    c.out.value = Amount(decompress_amount(read_varint(r)));
    const u64 n = read_varint(r);
    if (n < kSpecialScripts) {
        const size_t len = n < 2 ? 20 : 32;
        const u8* p = r.take(len);
        c.out.script_pubkey = decompress_script(n, Bytes(p, p + len));
    } else {
        const u64 len = n - kSpecialScripts;
        if (len > kMaxScriptSize) {  // unspendable: OP_RETURN, data skipped
            r.take(size_t(len));
            c.out.script_pubkey = {0x6a};
        } else {
            const u8* p = r.take(size_t(len));
            c.out.script_pubkey.assign(p, p + len);
        }
    }
    return c;
}

}  // namespace

Bytes serialize_coin_db(const Coin& c) {
    Writer w;
    write_varint(w, u64(c.height) * 2 + (c.coinbase ? 1 : 0));
    write_varint(w, compress_amount(u64(c.out.value)));
    Bytes comp;
    if (compress_script(c.out.script_pubkey, comp)) {
        w.raw(comp);
    } else {
        write_varint(w, c.out.script_pubkey.size() + kSpecialScripts);
        w.raw(c.out.script_pubkey);
    }
    return std::move(w.buf);
}

bool deserialize_coin_db(const u8* p, size_t n, Coin& c) {
    try {
        Reader r(p, n);
        const u64 code = read_varint(r);
        c.height = u32(code >> 1);
        c.coinbase = code & 1;
        c.out.value = Amount(decompress_amount(read_varint(r)));
        const u64 k = read_varint(r);
        if (k < kSpecialScripts) {
            const size_t len = k < 2 ? 20 : 32;
            const u8* q = r.take(len);
            c.out.script_pubkey = decompress_script(k, Bytes(q, q + len));
            if (c.out.script_pubkey.empty()) return false;  // an invalid compressed key
        } else {
            const u64 len = k - kSpecialScripts;
            if (len > kMaxScriptSize) {  // stored unspendable: OP_RETURN, data skipped
                r.take(size_t(len));
                c.out.script_pubkey = {0x6a};
            } else {
                const u8* q = r.take(size_t(len));
                c.out.script_pubkey.assign(q, q + len);
            }
        }
        return true;
    } catch (const std::exception&) {
        return false;
    }
}

void append_varint(Bytes& out, u64 n) {
    Writer w;
    write_varint(w, n);
    out.insert(out.end(), w.buf.begin(), w.buf.end());
}

bool parse_varint(const u8*& p, const u8* end, u64& n) {
    try {
        Reader r(p, size_t(end - p));
        n = read_varint(r);
        p = end - r.remaining();
        return true;
    } catch (const std::exception&) {
        return false;
    }
}

u64 compress_amount(u64 n) {
    if (n == 0) return 0;
    int e = 0;
    while ((n % 10) == 0 && e < 9) {
        n /= 10;
        ++e;
    }
    if (e < 9) {
        const int d = int(n % 10);
        n /= 10;
        return 1 + (n * 9 + u64(d) - 1) * 10 + u64(e);
    }
    return 1 + (n - 1) * 10 + 9;
}

u64 decompress_amount(u64 x) {
    if (x == 0) return 0;
    --x;
    int e = int(x % 10);
    x /= 10;
    u64 n;
    if (e < 9) {
        const int d = int(x % 9) + 1;
        x /= 9;
        n = x * 10 + u64(d);
    } else {
        n = x + 1;
    }
    while (e--) n *= 10;
    return n;
}

Bytes serialize_block_undo(const BlockUndo& u) {
    Writer w;
    w.compact_size(u.vtxundo.size());
    for (auto& t : u.vtxundo) {
        w.compact_size(t.prev.size());
        for (auto& c : t.prev) write_coin_undo(w, c);
    }
    return w.buf;
}

BlockUndo deserialize_block_undo(const Bytes& b) {
    Reader r(b);
    BlockUndo u;
    u.vtxundo.resize(size_t(r.compact_size()));
    for (auto& t : u.vtxundo) {
        t.prev.resize(size_t(r.compact_size()));
        for (auto& c : t.prev) c = read_coin_undo(r);
    }
    if (!r.empty()) throw std::runtime_error("trailing data after block undo");
    return u;
}

// ------------------------------------------------------------------ sigops
namespace {

// the last data push of a push-only scriptSig (the P2SH redeem script), or false
bool last_push(const Bytes& script_sig, Bytes& data) {
    size_t pc = 0;
    u8 op;
    Bytes d;
    data.clear();
    while (pc < script_sig.size()) {
        if (!script_get_op(script_sig, pc, op, &d)) return false;
        if (op > 0x60) return false;  // OP_16
        data = d;
    }
    return true;
}

int64_t witness_sigops(int version, const Bytes& program, const std::vector<Bytes>& witness) {
    if (version != 0) return 0;
    if (program.size() == 20) return 1;
    if (program.size() == 32 && !witness.empty()) return script_sigop_count(witness.back(), true);
    return 0;
}

}  // namespace

int64_t tx_legacy_sigops(const Transaction& tx) {
    int64_t legacy = 0;
    for (auto& in : tx.vin) legacy += script_sigop_count(in.script_sig, false);
    for (auto& o : tx.vout) legacy += script_sigop_count(o.script_pubkey, false);
    return legacy;
}

int64_t tx_sigop_cost(const Transaction& tx, const std::vector<const Coin*>& spent, u32 flags) {
    int64_t cost = tx_legacy_sigops(tx) * 4;
    if (tx.is_coinbase()) return cost;
    if (spent.size() != tx.vin.size()) throw std::invalid_argument("tx_sigop_cost: one spent coin per input");
    for (size_t i = 0; i < tx.vin.size(); ++i) {
        const Bytes& spk = spent[i]->out.script_pubkey;
        const TxIn& in = tx.vin[i];
        Bytes redeem;
        const bool p2sh = script_is_p2sh(spk) && last_push(in.script_sig, redeem);
        if ((flags & SCRIPT_VERIFY_P2SH) && p2sh) cost += int64_t(script_sigop_count(redeem, true)) * 4;
        if (flags & SCRIPT_VERIFY_WITNESS) {
            int v;
            Bytes prog;
            if (script_is_witness_program(spk, v, prog)) cost += witness_sigops(v, prog, in.witness);
            else if (p2sh && script_is_witness_program(redeem, v, prog)) cost += witness_sigops(v, prog, in.witness);
        }
    }
    return cost;
}

// ------------------------------------------------------------------ connect / disconnect
bool verify_input_host(const Transaction& tx, unsigned n_in, const Coin& coin, u32 flags, ScriptError* err) {
    const PrecomputedTx cache(tx);
    const TxSigChecker checker(&tx, n_in, coin.out.value, &cache);
    return verify_script(tx.vin[n_in].script_sig, coin.out.script_pubkey, &tx.vin[n_in].witness, flags, checker, err);
}

namespace {

bool is_unspendable(const Bytes& spk) { return assets::script_unspendable(spk); }

}  // namespace

ConnectResult connect_block(const Block& block, int height, CoinsView& view, const ConnectOptions& opt,
                            BlockUndo& undo) {
    ConnectResult res;
    undo.vtxundo.clear();
    std::vector<OutPoint> added;
    const size_t asset_mark = opt.assets ? opt.assets->mark() : 0;
    auto fail = [&](const std::string& reason, int dos) {
        if (opt.assets) opt.assets->rollback_to(asset_mark);
        // roll back: restore what the block spent (later transactions first), then drop every
        // output it added (that also removes in-block outputs the restore just put back)
        for (size_t t = undo.vtxundo.size(); t-- > 0;) {
            const Transaction& tx = block.vtx[t + 1];
            for (size_t i = 0; i < undo.vtxundo[t].prev.size(); ++i)
                view.add(tx.vin[i].prevout, undo.vtxundo[t].prev[i]);
        }
        for (auto it = added.rbegin(); it != added.rend(); ++it) view.spend(*it);
        undo.vtxundo.clear();
        res.ok = false;
        res.reject = reason;
        res.dos = dos;
        res.sigs.clear();
        res.sig_at.clear();
        return res;
    };
    struct Check {
        u32 t, i;
        Amount value;
        Bytes spk;
        bool ok = true;
        ScriptError err = ScriptError::OK;
        std::vector<PendingSig> sigs;
    };
    std::vector<Check> checks;
    std::vector<std::unique_ptr<PrecomputedTx>> caches(block.vtx.size());
    for (size_t t = 0; t < block.vtx.size(); ++t) {
        const Transaction& tx = block.vtx[t];
        const Uint256 txid = tx.txid();
        std::vector<const Coin*> spent;
        if (!tx.is_coinbase()) {
            Amount in_sum = 0;
            std::vector<int> prev_heights;
            for (auto& in : tx.vin) {
                const Coin* c = view.find(in.prevout);
                if (!c) return fail("bad-txns-inputs-missingorspent", 100);
                if (c->coinbase && height - int(c->height) < kCoinbaseMaturity)
                    return fail("bad-txns-premature-spend-of-coinbase", 0);
                if (c->out.value < 0 || c->out.value > kMaxMoney) return fail("bad-txns-inputvalues-outofrange", 100);
                in_sum += c->out.value;
                if (in_sum < 0 || in_sum > kMaxMoney) return fail("bad-txns-inputvalues-outofrange", 100);
                spent.push_back(c);
                prev_heights.push_back(int(c->height));
            }
            const Amount out_sum = tx.value_out();
            if (in_sum < out_sum) return fail("bad-txns-in-belowout", 100);
            const Amount fee = in_sum - out_sum;
            res.fees += fee;
            if (res.fees < 0 || res.fees > kMaxMoney) return fail("bad-txns-accumulated-fee-outofrange", 100);
            if (opt.assets) {
                if (!opt.asset_flags.assets) {
                    for (auto& o : tx.vout) {
                        if (assets::asset_script_kind(o.script_pubkey) != assets::OutKind::NONE)
                            return fail("bad-txns-assets-not-active", 100);
                        if (assets::null_kind(o.script_pubkey) != assets::NullKind::NONE)
                            return fail("bad-txns-null-data-assets-not-active", 100);
                    }
                } else {
                    const std::string why = assets::check_tx_contextual(tx, spent, *opt.assets, opt.asset_flags);
                    if (!why.empty()) return fail(why, 100);
                }
            }
            // BIP68 relative lock-times (CalculateSequenceLocks / EvaluateSequenceLocks)
            if (opt.sequence_locks && (opt.script_flags & SCRIPT_VERIFY_CHECKSEQUENCEVERIFY) && u32(tx.version) >= 2) {
                int min_height = -1;
                int64_t min_time = -1;
                for (size_t i = 0; i < tx.vin.size(); ++i) {
                    const u32 seq = tx.vin[i].sequence;
                    if (seq & (1u << 31)) continue;
                    if (seq & (1u << 22)) {
                        const int64_t coin_time = opt.mtp_at ? opt.mtp_at(std::max(prev_heights[i] - 1, 0)) : 0;
                        min_time = std::max(min_time, coin_time + (int64_t(seq & 0xffff) << 9) - 1);
                    } else {
                        min_height = std::max(min_height, prev_heights[i] + int(seq & 0xffff) - 1);
                    }
                }
                if (min_height >= height || min_time >= opt.block_mtp) return fail("bad-txns-nonfinal", 100);
            }
        }
        res.sigop_cost += tx_sigop_cost(tx, spent, opt.script_flags);
        if (res.sigop_cost > kMaxBlockSigopsCost) return fail("bad-blk-sigops", 100);
        if (!tx.is_coinbase() && opt.check_scripts) {
            caches[t] = std::make_unique<PrecomputedTx>(tx);
            for (size_t i = 0; i < tx.vin.size(); ++i)
                checks.push_back({u32(t), u32(i), spent[i]->out.value, spent[i]->out.script_pubkey});
        }
        // spend the inputs, recording them for undo
        if (!tx.is_coinbase()) {
            TxUndo tu;
            tu.prev.reserve(tx.vin.size());
            for (auto& in : tx.vin) {
                Coin c;
                view.spend(in.prevout, &c);
                tu.prev.push_back(std::move(c));
            }
            undo.vtxundo.push_back(std::move(tu));
        }
        for (u32 n = 0; n < tx.vout.size(); ++n) {
            if (is_unspendable(tx.vout[n].script_pubkey)) continue;
            OutPoint o;
            o.hash = txid;
            o.n = n;
            if (view.find(o)) return fail("bad-txns-BIP30", 100);  // would overwrite an unspent output
            Coin c;
            c.out = tx.vout[n];
            c.height = u32(height);
            c.coinbase = tx.is_coinbase();
            view.add(o, std::move(c));
            added.push_back(o);
        }
        if (opt.assets && opt.asset_flags.assets) {
            static const std::vector<Coin> kNoCoins;
            assets::apply_tx(tx, tx.is_coinbase() ? kNoCoins : undo.vtxundo.back().prev, height, opt.block_hash,
                             *opt.assets);
        }
    }
    // the script checks (CCheckQueue): inline, or spread over worker threads
    auto run = [&](Check& c) {
        const Transaction& tx = block.vtx[c.t];
        TxSigChecker checker(&tx, c.i, c.value, caches[c.t].get());
        if (opt.defer_sigs) checker.pending = &c.sigs;
        if (opt.sigcache) checker.sigcache = TxSigChecker::CacheMode::USE;
        c.ok = verify_script(tx.vin[c.i].script_sig, c.spk, &tx.vin[c.i].witness, opt.script_flags, checker, &c.err);
    };
    const int nthreads = std::max(1, std::min<int>(opt.threads, int(checks.size() / 16)));
    if (nthreads <= 1) {
        for (auto& c : checks) {
            run(c);
            if (!c.ok) break;
        }
    } else {
        std::atomic<size_t> next{0};
        std::atomic<size_t> first_bad{checks.size()};
        auto worker = [&] {
            for (size_t k; (k = next.fetch_add(1, std::memory_order_relaxed)) < checks.size();) {
                if (k > first_bad.load(std::memory_order_relaxed)) break;  // a prior input already failed
                run(checks[k]);
                if (!checks[k].ok) {
                    size_t cur = first_bad.load();
                    while (k < cur && !first_bad.compare_exchange_weak(cur, k)) {}
                }
            }
        };
        std::vector<std::thread> pool;
        for (int w = 1; w < nthreads; ++w) pool.emplace_back(worker);
        worker();
        for (auto& th : pool) th.join();
    }
    for (auto& c : checks) {
        if (!c.ok)
            return fail(std::string("mandatory-script-verify-flag-failed (") + script_error_name(c.err) + ")", 100);
        for (auto& p : c.sigs) {
            res.sigs.push_back(std::move(p));
            res.sig_at.emplace_back(c.t, c.i);
        }
    }
    if (opt.assets) {
        res.asset_undo = opt.assets->journal_since(asset_mark);
        opt.assets->clear_journal();  // the record now lives with the caller (asset undo store)
    }
    return res;
}

bool disconnect_block(const Block& block, const BlockUndo& undo, CoinsView& view, assets::State* assets,
                      const Bytes* asset_undo) {
    if (undo.vtxundo.size() + 1 != block.vtx.size()) return false;
    bool clean = true;
    if (assets && asset_undo && !asset_undo->empty() && !assets->undo(*asset_undo)) clean = false;
    for (size_t t = block.vtx.size(); t-- > 0;) {
        const Transaction& tx = block.vtx[t];
        const Uint256 txid = tx.txid();
        for (u32 n = 0; n < tx.vout.size(); ++n) {
            if (is_unspendable(tx.vout[n].script_pubkey)) continue;
            OutPoint o;
            o.hash = txid;
            o.n = n;
            if (!view.spend(o)) clean = false;
        }
        if (t == 0) break;
        const TxUndo& tu = undo.vtxundo[t - 1];
        if (tu.prev.size() != tx.vin.size()) return false;
        for (size_t i = tx.vin.size(); i-- > 0;) {
            if (view.find(tx.vin[i].prevout)) clean = false;
            view.add(tx.vin[i].prevout, tu.prev[i]);
        }
    }
    return clean;
}

}  // namespace nodexa
