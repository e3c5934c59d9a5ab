// HeaderBatch: see headerbatch.hpp.
#include "headerbatch.hpp"

#include <cstring>

#include "../util/workpool.hpp"

namespace nodexa {

HeaderBatch HeaderBatch::from_bytes(const u8* data, size_t len, u32 act, std::shared_ptr<const void> keep) {
    HeaderBatch b;
    b.act = act;
    b.keep_ = std::move(keep);
    b.src_ = b.keep_ ? data : nullptr;
    // one cheap serial scan for the record boundaries (80 / 120 / extended by version bit and
    // nTime) and the Equihash records; everything else is one parallel pass over the wire bytes
    std::vector<size_t>& off = b.off_;
    off.reserve(len / 120 + 2);
    std::vector<u32> sol_at;  // offset of each Equihash solution within its record
    size_t o = 0;
    while (o < len) {
        if (len - o < 80) throw std::out_of_range("HeaderBatch: truncated header");
        const u32 version = load_le32(data + o);
        const u32 time = load_le32(data + o + 68);
        if (version & u32(kEquihashVersionBit)) {
            if (len - o < 112) throw std::out_of_range("HeaderBatch: truncated header");
            Reader r(data + o + 112, len - o - 112);
            const u64 sol = r.compact_size();
            if (sol > 4096) throw std::runtime_error("equihash solution too large");
            b.eq_index.push_back(u32(off.size()));
            sol_at.push_back(u32(sol == 1344 ? 112 + r.pos() : 0));
            off.push_back(o);
            o += 112 + r.pos() + sol;
        } else {
            off.push_back(o);
            o += time < act ? 80 : 120;
        }
    }
    if (o != len) throw std::out_of_range("HeaderBatch: truncated header");
    const size_t n = off.size();
    off.push_back(len);
    b.n_ = n;
    b.materialized_ = false;
    if (!b.keep_) b.raw_.resize(len);
    b.kinds.resize(n);
    b.rows.resize(n * kBatchRow);
    const size_t m = b.eq_index.size();
    b.eq_ser_len = m ? off[b.eq_index[0] + 1] - off[b.eq_index[0]] : 0;
    b.eq_msgs.assign(m * 128, '\0');
    b.eq_sols.assign(m * 1344, '\0');
    b.eq_ser.resize(m * b.eq_ser_len);
    bool uniform = true;
    for (size_t k = 0; k < m; ++k) {
        const size_t i = b.eq_index[k];
        uniform = uniform && sol_at[k] != 0 && off[i + 1] - off[i] == b.eq_ser_len;
    }
    b.eq_uniform = uniform;
    char* raw = b.keep_ ? nullptr : b.raw_.data();
    parallel_for_each(n, [&](size_t i) {
        const u8* src = data + off[i];
        const size_t rl = off[i + 1] - off[i];
        if (raw) std::memcpy(raw + off[i], src, rl);
        u8* row = reinterpret_cast<u8*>(&b.rows[i * kBatchRow]);
        const bool eq = load_le32(src) & u32(kEquihashVersionBit);
        const size_t keep = eq ? 80 : rl;  // nHeight sits at bytes 76..79 of the Equihash prefix
        std::memcpy(row, src, keep);
        std::memset(row + keep, 0, kBatchRow - keep);
        b.kinds[i] = eq ? 2 : rl == 80 ? 3 : 0;
    }, 512);
    parallel_for_each(m, [&](size_t k) {
        const size_t i = b.eq_index[k];
        const u8* src = data + off[i];
        std::memcpy(&b.eq_msgs[k * 128], src, 112);  // CKAWPOWInput (80 bytes) + nNonce256
        if (sol_at[k]) std::memcpy(&b.eq_sols[k * 1344], src + sol_at[k], 1344);
        if (off[i + 1] - off[i] == b.eq_ser_len) std::memcpy(&b.eq_ser[k * b.eq_ser_len], src, b.eq_ser_len);
    }, 16);
    return b;
}

BlockHeader HeaderBatch::header(size_t i) {
    std::lock_guard<std::mutex> lk(*mu_);
    if (i >= n_) throw std::out_of_range("HeaderBatch: index out of range");
    if (materialized_) return hs[i];
    const u8* raw = keep_ ? src_ : reinterpret_cast<const u8*>(raw_.data());
    Reader r(raw + off_[i], off_[i + 1] - off_[i]);
    return BlockHeader::deserialize(r, act);
}

void HeaderBatch::materialize() {
    std::lock_guard<std::mutex> lk(*mu_);
    if (materialized_) return;
    hs.resize(n_);
    const u8* raw = keep_ ? src_ : reinterpret_cast<const u8*>(raw_.data());
    parallel_for_each(n_, [&](size_t i) {
        Reader r(raw + off_[i], off_[i + 1] - off_[i]);
        hs[i] = BlockHeader::deserialize(r, act);
    }, 512);
    materialized_ = true;
}

HeaderBatch HeaderBatch::from_headers(std::vector<BlockHeader> headers, u32 act) {
    HeaderBatch b;
    b.act = act;
    b.hs = std::move(headers);
    b.n_ = b.hs.size();
    b.pack();
    return b;
}

void HeaderBatch::pack() {
    const size_t n = hs.size();
    kinds.assign(n, '\0');
    rows.assign(n * kBatchRow, '\0');  // (the object path fills only the fields it writes)
    eq_index.clear();
    for (size_t i = 0; i < n; ++i)
        if (hs[i].is_equihash()) eq_index.push_back(u32(i));
    const size_t m = eq_index.size();
    eq_msgs.assign(m * 128, '\0');
    eq_sols.assign(m * 1344, '\0');
    eq_ser_len = m ? hs[eq_index[0]].bytes(act).size() : 0;
    eq_ser.assign(m * eq_ser_len, '\0');
    parallel_for_each(n, [&](size_t i) {
        const BlockHeader& h = hs[i];
        u8* row = reinterpret_cast<u8*>(&rows[i * kBatchRow]);
        // the 76 bytes every header kind starts with, then its own tail (no per-header allocation)
        store_le32(row, u32(h.version));
        std::memcpy(row + 4, h.prev.data, 32);
        std::memcpy(row + 36, h.merkle_root.data, 32);
        store_le32(row + 68, h.time);
        store_le32(row + 72, h.bits);
        if (h.is_equihash()) {
            kinds[i] = 2;
            store_le32(row + 76, h.height);  // the CKAWPOWInput prefix of the Equihash input
        } else if (!h.is_kawpow(act)) {
            kinds[i] = 3;
            store_le32(row + 76, h.nonce);   // the 80-byte legacy header
        } else {
            store_le32(row + 76, h.height);  // the 120-byte KawPow header
            store_le64(row + 80, h.nonce64);
            std::memcpy(row + 88, h.mix_hash.data, 32);
        }
    }, 512);
    // the Equihash inputs, solutions and serializations (1.5 KB each) on all cores too
    std::vector<u8> ok(m, 1);
    parallel_for_each(m, [&](size_t k) {
        const BlockHeader& h = hs[eq_index[k]];
        const Bytes in = h.equihash_input();
        std::memcpy(&eq_msgs[k * 128], in.data(), std::min<size_t>(in.size(), 128));
        if (h.solution.size() == 1344)
            std::memcpy(&eq_sols[k * 1344], h.solution.data(), 1344);
        else
            ok[k] = 0;
        const Bytes s = h.bytes(act);
        if (s.size() == eq_ser_len)
            std::memcpy(&eq_ser[k * eq_ser_len], s.data(), s.size());
        else
            ok[k] = 0;
    }, 16);
    bool uniform = true;
    for (u8 x : ok) uniform = uniform && x;
    eq_uniform = uniform;
}

}  // namespace nodexa
