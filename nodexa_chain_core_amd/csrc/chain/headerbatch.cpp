// HeaderBatch: see headerbatch.hpp.
#include "headerbatch.hpp"

#include <cstring>

#include "../util/workpool.hpp"

namespace nodexa {

HeaderBatch HeaderBatch::from_bytes(const u8* data, size_t len, u32 act) {
    HeaderBatch b;
    b.act = act;
    // one cheap serial scan for the record boundaries (80 / 120 / extended by version bit and
    // nTime), then every header is decoded in parallel straight from the caller's buffer
    std::vector<size_t> off;
    off.reserve(len / 120 + 1);
    size_t o = 0;
    while (o < len) {
        if (len - o < 80) throw std::out_of_range("HeaderBatch: truncated header");
        off.push_back(o);
        const u32 version = load_le32(data + o);
        const u32 time = load_le32(data + o + 68);
        if (version & u32(kEquihashVersionBit)) {
            Reader r(data + o + 112, len - std::min(len, o + 112));
            const u64 sol = r.compact_size();
            o += 112 + r.pos() + sol;
        } else {
            o += time < act ? 80 : 120;
        }
    }
    if (o != len) throw std::out_of_range("HeaderBatch: truncated header");
    b.hs.resize(off.size());
    parallel_for_each(off.size(), [&](size_t i) {
        const size_t end = i + 1 < off.size() ? off[i + 1] : len;
        Reader r(data + off[i], end - off[i]);
        b.hs[i] = BlockHeader::deserialize(r, act);
    }, 512);
    b.pack();
    return b;
}

HeaderBatch HeaderBatch::from_headers(std::vector<BlockHeader> headers, u32 act) {
    HeaderBatch b;
    b.act = act;
    b.hs = std::move(headers);
    b.pack();
    return b;
}

void HeaderBatch::pack() {
    const size_t n = hs.size();
    kinds.assign(n, '\0');
    rows.assign(n * kBatchRow, '\0');
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
