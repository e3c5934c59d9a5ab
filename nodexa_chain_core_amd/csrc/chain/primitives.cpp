#include "primitives.hpp"

#include "../crypto/sha256.hpp"

namespace nodexa {

namespace {
Uint256 sha256d_u(const Bytes& b) {
    Uint256 u;
    sha256d(b.data(), b.size(), u.data);
    return u;
}
}  // namespace

void Transaction::serialize(Writer& w, bool with_witness) const {
    const bool wit = with_witness && has_witness();
    w.i32_(version);
    if (wit) {
        w.u8_(0x00);  // marker (empty vin)
        w.u8_(0x01);  // flags
    }
    w.compact_size(vin.size());
    for (auto& in : vin) {
        w.u256(in.prevout.hash);
        w.u32_(in.prevout.n);
        w.var_bytes(in.script_sig);
        w.u32_(in.sequence);
    }
    w.compact_size(vout.size());
    for (auto& out : vout) {
        w.i64_(out.value);
        w.var_bytes(out.script_pubkey);
    }
    if (wit) {
        for (auto& in : vin) {
            w.compact_size(in.witness.size());
            for (auto& item : in.witness) w.var_bytes(item);
        }
    }
    w.u32_(lock_time);
}

Transaction Transaction::deserialize(Reader& r, bool allow_witness) {
    Transaction tx;
    tx.version = r.i32_();
    u8 flags = 0;
    auto read_vin = [&] {
        const u64 n = r.compact_size();
        tx.vin.resize(size_t(n));
        for (auto& in : tx.vin) {
            in.prevout.hash = r.u256();
            in.prevout.n = r.u32_();
            in.script_sig = r.var_bytes();
            in.sequence = r.u32_();
        }
    };
    auto read_vout = [&] {
        const u64 n = r.compact_size();
        tx.vout.resize(size_t(n));
        for (auto& out : tx.vout) {
            out.value = r.i64_();
            out.script_pubkey = r.var_bytes();
        }
    };
    read_vin();
    if (tx.vin.empty() && allow_witness) {
        flags = r.u8_();
        if (flags != 0) {
            read_vin();
            read_vout();
        }
    } else {
        read_vout();
    }
    if ((flags & 1) && allow_witness) {
        flags ^= 1;
        for (auto& in : tx.vin) {
            const u64 n = r.compact_size();
            in.witness.resize(size_t(n));
            for (auto& item : in.witness) item = r.var_bytes();
        }
        if (!tx.has_witness()) throw std::runtime_error("Superfluous witness record");
    }
    if (flags) throw std::runtime_error("Unknown transaction optional data");
    tx.lock_time = r.u32_();
    return tx;
}

Uint256 Transaction::txid() const { return sha256d_u(bytes(false)); }
Uint256 Transaction::wtxid() const { return sha256d_u(bytes(true)); }

void BlockHeader::serialize(Writer& w, u32 act) const {
    w.i32_(version);
    w.u256(prev);
    w.u256(merkle_root);
    w.u32_(time);
    w.u32_(bits);
    if (is_equihash()) {
        w.u32_(height);
        w.u256(nonce256);
        w.var_bytes(solution);
    } else if (time < act) {
        w.u32_(nonce);
    } else {
        w.u32_(height);
        w.u64_(nonce64);
        w.u256(mix_hash);
    }
}

Bytes BlockHeader::equihash_input() const {
    Bytes b = kawpow_input();
    b.insert(b.end(), nonce256.data, nonce256.data + 32);
    return b;
}

Uint256 BlockHeader::equihash_hash(u32 act) const { return sha256d_u(bytes(act)); }

BlockHeader BlockHeader::deserialize(Reader& r, u32 act) {
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
        if (h.solution.size() > 4096) throw std::runtime_error("equihash solution too large");
    } else if (h.time < act) {
        h.nonce = r.u32_();
    } else {
        h.height = r.u32_();
        h.nonce64 = r.u64_();
        h.mix_hash = r.u256();
    }
    return h;
}

Bytes BlockHeader::legacy80() const {
    Writer w;
    w.i32_(version);
    w.u256(prev);
    w.u256(merkle_root);
    w.u32_(time);
    w.u32_(bits);
    w.u32_(nonce);
    return w.buf;
}

Bytes BlockHeader::kawpow_input() const {
    Writer w;
    w.i32_(version);
    w.u256(prev);
    w.u256(merkle_root);
    w.u32_(time);
    w.u32_(bits);
    w.u32_(height);
    return w.buf;
}

Uint256 BlockHeader::kawpow_header_hash() const { return sha256d_u(kawpow_input()); }

void Block::serialize(Writer& w, u32 act, bool with_witness) const {
    header.serialize(w, act);
    w.compact_size(vtx.size());
    for (auto& tx : vtx) tx.serialize(w, with_witness);
}

Block Block::deserialize(Reader& r, u32 act) {
    Block b;
    b.header = BlockHeader::deserialize(r, act);
    const u64 n = r.compact_size();
    b.vtx.reserve(size_t(n));
    for (u64 i = 0; i < n; ++i) b.vtx.push_back(Transaction::deserialize(r));
    return b;
}

Uint256 compute_merkle_root(std::vector<Uint256> hashes, bool* mutated) {
    bool mutation = false;
    if (hashes.empty()) {
        if (mutated) *mutated = false;
        return Uint256();
    }
    while (hashes.size() > 1) {
        if (mutated)
            for (size_t pos = 0; pos + 1 < hashes.size(); pos += 2)
                if (hashes[pos] == hashes[pos + 1]) mutation = true;
        if (hashes.size() & 1) hashes.push_back(hashes.back());
        std::vector<Uint256> next(hashes.size() / 2);
        for (size_t i = 0; i < next.size(); ++i) sha256d_64(hashes[2 * i].data, hashes[2 * i + 1].data, next[i].data);
        hashes.swap(next);
    }
    if (mutated) *mutated = mutation;
    return hashes[0];
}

Uint256 block_merkle_root(const Block& b, bool* mutated) {
    std::vector<Uint256> leaves;
    leaves.reserve(b.vtx.size());
    for (auto& tx : b.vtx) leaves.push_back(tx.txid());
    return compute_merkle_root(std::move(leaves), mutated);
}

Uint256 block_witness_merkle_root(const Block& b, bool* mutated) {
    std::vector<Uint256> leaves;
    leaves.reserve(b.vtx.size());
    leaves.emplace_back();  // coinbase wtxid is 0
    for (size_t i = 1; i < b.vtx.size(); ++i) leaves.push_back(b.vtx[i].wtxid());
    return compute_merkle_root(std::move(leaves), mutated);
}

int witness_commitment_index(const Block& b) {
    int pos = -1;
    if (b.vtx.empty()) return -1;
    const auto& cb = b.vtx[0];
    for (size_t o = 0; o < cb.vout.size(); ++o) {
        const Bytes& s = cb.vout[o].script_pubkey;
        if (s.size() >= 38 && s[0] == 0x6a && s[1] == 0x24 && s[2] == 0xaa && s[3] == 0x21 && s[4] == 0xa9 &&
            s[5] == 0xed)
            pos = int(o);
    }
    return pos;
}

}  // namespace nodexa
