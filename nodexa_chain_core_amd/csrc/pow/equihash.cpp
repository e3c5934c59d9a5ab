#include "equihash.hpp"

#include <algorithm>
#include <array>
#include <functional>
#include <thread>

namespace nodexa {

void EquihashParams::personal(u8 out[16]) const {
    std::memcpy(out, "ZcashPoW", 8);
    store_le32(out + 8, u32(n));
    store_le32(out + 12, u32(k));
}

Blake2b equihash_base_state(const EquihashParams& p, const u8* input, size_t n) {
    u8 pers[16];
    p.personal(pers);
    Blake2b s(size_t(p.digest_bytes()), pers);
    s.update(input, n);
    return s;
}

void equihash_leaf(const EquihashParams& p, const Blake2b& base, u32 i, u8* out) {
    Blake2b s = base;
    u8 le[4];
    store_le32(le, i / u32(p.indices_per_hash()));
    s.update(le, 4);
    u8 digest[64];
    s.final(digest);
    std::memcpy(out, digest + (i % u32(p.indices_per_hash())) * p.hash_bytes(), size_t(p.hash_bytes()));
}

Bytes equihash_pack_indices(const EquihashParams& p, const std::vector<u32>& idx) {
    const int bits = p.collision_bits() + 1;
    Bytes out(size_t((idx.size() * bits + 7) / 8), 0);
    size_t bitpos = 0;
    for (u32 v : idx) {
        for (int b = bits - 1; b >= 0; --b, ++bitpos)
            if ((v >> b) & 1) out[bitpos / 8] |= u8(0x80 >> (bitpos % 8));
    }
    return out;
}

std::vector<u32> equihash_unpack_indices(const EquihashParams& p, const Bytes& sol) {
    const int bits = p.collision_bits() + 1;
    const size_t count = sol.size() * 8 / bits;
    std::vector<u32> out(count, 0);
    size_t bitpos = 0;
    for (size_t i = 0; i < count; ++i)
        for (int b = 0; b < bits; ++b, ++bitpos)
            out[i] = (out[i] << 1) | ((sol[bitpos / 8] >> (7 - bitpos % 8)) & 1);
    return out;
}

namespace {

using Row = std::array<u64, 4>;  // n-bit string, big-endian, zero padded to 256 bits

Row load_row(const u8* b, int nbytes) {
    u8 tmp[32] = {0};
    std::memcpy(tmp, b, size_t(nbytes));
    return Row{load_be64(tmp), load_be64(tmp + 8), load_be64(tmp + 16), load_be64(tmp + 24)};
}

inline u64 bits_at(const Row& w, int off, int len) {
    const int wi = off / 64, bo = off % 64;
    const unsigned __int128 x = ((unsigned __int128)w[wi] << 64) | (wi + 1 < 4 ? w[wi + 1] : 0);
    return u64(x >> (128 - bo - len)) & ((len == 64) ? ~0ULL : ((1ULL << len) - 1));
}

inline bool zero_from(const Row& w, int off) {
    // bits [off, 256) all zero
    const int wi = off / 64, bo = off % 64;
    if (bo) {
        if (w[wi] & (~0ULL >> bo)) return false;
    } else if (w[wi]) {
        return false;
    }
    for (int i = wi + 1; i < 4; ++i)
        if (w[i]) return false;
    return true;
}

Row xor_rows(const Row& a, const Row& b) { return Row{a[0] ^ b[0], a[1] ^ b[1], a[2] ^ b[2], a[3] ^ b[3]}; }

}  // namespace

bool equihash_verify(const EquihashParams& p, const u8* input, size_t n, const std::vector<u32>& indices,
                     std::string* reason) {
    auto fail = [&](const char* r) {
        if (reason) *reason = r;
        return false;
    };
    if (int(indices.size()) != p.solution_indices()) return fail("bad-size");
    for (u32 v : indices)
        if (v >= p.num_leaves()) return fail("index-range");
    const Blake2b base = equihash_base_state(p, input, n);
    struct Node {
        Row h;
        std::vector<u32> idx;
    };
    std::vector<Node> rows(indices.size());
    u8 leaf[64];
    for (size_t i = 0; i < indices.size(); ++i) {
        equihash_leaf(p, base, indices[i], leaf);
        rows[i].h = load_row(leaf, p.hash_bytes());
        rows[i].idx = {indices[i]};
    }
    const int cb = p.collision_bits();
    for (int level = 1; level <= p.k; ++level) {
        std::vector<Node> next(rows.size() / 2);
        for (size_t j = 0; j < next.size(); ++j) {
            const Node& a = rows[2 * j];
            const Node& b = rows[2 * j + 1];
            const Row x = xor_rows(a.h, b.h);
            // the first level*cb bits (all n bits at the root) must be zero
            const int zero_bits = (level < p.k) ? level * cb : p.n;
            bool ok = true;
            for (int off = 0; off < zero_bits && ok; off += 32) ok = bits_at(x, off, std::min(32, zero_bits - off)) == 0;
            if (!ok) return fail(level < p.k ? "collision" : "nonzero");
            if (a.idx.front() >= b.idx.front()) return fail("order");
            next[j].h = x;
            next[j].idx = a.idx;
            next[j].idx.insert(next[j].idx.end(), b.idx.begin(), b.idx.end());
        }
        rows.swap(next);
    }
    std::vector<u32> sorted = indices;
    std::sort(sorted.begin(), sorted.end());
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end()) return fail("duplicate");
    if (reason) reason->clear();
    return true;
}

std::vector<std::vector<u32>> equihash_solve_cpu(const EquihashParams& p, const u8* input, size_t n,
                                                 size_t max_solutions, EquihashSolveStats* stats, int threads) {
    const u32 N = p.num_leaves();
    const int cb = p.collision_bits();
    const Blake2b base = equihash_base_state(p, input, n);
    if (threads <= 0) threads = int(std::max(1u, std::thread::hardware_concurrency()));

    // ---- round 0: rows from BLAKE2b (one digest serves indices_per_hash leaves)
    std::vector<Row> hashes(N);
    {
        const u32 per = u32(p.indices_per_hash());
        const u32 digests = N / per;
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t)
            pool.emplace_back([&, t] {
                u8 le[4], digest[64];
                for (u32 g = u32(t); g < digests; g += u32(threads)) {
                    Blake2b s = base;
                    store_le32(le, g);
                    s.update(le, 4);
                    s.final(digest);
                    for (u32 j = 0; j < per; ++j) hashes[g * per + j] = load_row(digest + j * p.hash_bytes(), p.hash_bytes());
                }
            });
        for (auto& th : pool) th.join();
    }

    // refs[level][row] = (a, b) into level-1 rows; level 0 rows are leaves.
    std::vector<std::vector<std::pair<u32, u32>>> refs(size_t(p.k));
    const size_t max_rows = size_t(N) * 2;
    std::vector<u32> count(size_t(1) << cb);
    std::vector<u32> order;
    for (int r = 1; r < p.k; ++r) {
        const size_t rows = hashes.size();
        if (stats) stats->rows_per_round.push_back(rows);
        std::fill(count.begin(), count.end(), 0);
        for (size_t i = 0; i < rows; ++i) ++count[size_t(bits_at(hashes[i], (r - 1) * cb, cb))];
        std::vector<u32> start(count.size() + 1, 0);
        for (size_t b = 0; b < count.size(); ++b) start[b + 1] = start[b] + count[b];
        order.assign(rows, 0);
        {
            std::vector<u32> fill(start.begin(), start.end() - 1);
            for (size_t i = 0; i < rows; ++i) order[fill[size_t(bits_at(hashes[i], (r - 1) * cb, cb))]++] = u32(i);
        }
        std::vector<Row> next;
        std::vector<std::pair<u32, u32>>& ref = refs[size_t(r)];
        next.reserve(rows + rows / 8);
        ref.reserve(rows + rows / 8);
        for (size_t b = 0; b < count.size() && next.size() < max_rows; ++b) {
            for (u32 x = start[b]; x < start[b + 1]; ++x)
                for (u32 y = x + 1; y < start[b + 1]; ++y) {
                    const u32 ia = order[x], ib = order[y];
                    const Row h = xor_rows(hashes[ia], hashes[ib]);
                    if (zero_from(h, r * cb)) {  // identical remainder: leads only to duplicate indices
                        if (stats) ++stats->discarded_duplicates;
                        continue;
                    }
                    next.push_back(h);
                    ref.emplace_back(ia, ib);
                }
        }
        hashes.swap(next);
    }
    if (stats) stats->rows_per_round.push_back(hashes.size());

    // ---- final round: collide on the last 2*cb bits
    std::vector<std::pair<u64, u32>> keyed(hashes.size());
    for (size_t i = 0; i < hashes.size(); ++i) keyed[i] = {bits_at(hashes[i], (p.k - 1) * cb, 2 * cb), u32(i)};
    std::sort(keyed.begin(), keyed.end());

    std::function<std::vector<u32>(int, u32)> expand = [&](int level, u32 row) -> std::vector<u32> {
        if (level == 0) return {row};
        const auto& pr = refs[size_t(level)][row];
        std::vector<u32> a = expand(level - 1, pr.first), b = expand(level - 1, pr.second);
        if (a.front() > b.front()) a.swap(b);
        a.insert(a.end(), b.begin(), b.end());
        return a;
    };

    std::vector<std::vector<u32>> sols;
    for (size_t x = 0; x < keyed.size() && sols.size() < max_solutions; ++x) {
        for (size_t y = x + 1; y < keyed.size() && keyed[y].first == keyed[x].first; ++y) {
            if (stats) ++stats->candidates;
            std::vector<u32> a = expand(p.k - 1, keyed[x].second), b = expand(p.k - 1, keyed[y].second);
            if (a.front() > b.front()) a.swap(b);
            a.insert(a.end(), b.begin(), b.end());
            std::vector<u32> s = a;
            std::sort(s.begin(), s.end());
            if (std::adjacent_find(s.begin(), s.end()) != s.end()) {
                if (stats) ++stats->discarded_duplicates;
                continue;
            }
            if (!equihash_verify(p, input, n, a)) continue;
            if (std::find(sols.begin(), sols.end(), a) == sols.end()) sols.push_back(std::move(a));
            if (sols.size() >= max_solutions) break;
        }
    }
    return sols;
}

}  // namespace nodexa
