// Berkeley DB btree reader and writer (see bdb.hpp for the page format).
#include "bdb.hpp"

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>
#include <stdexcept>
#include <utility>

#include <unistd.h>

namespace nodexa {
namespace bdb {
namespace {

constexpr uint32_t BTREE_MAGIC = 0x053162;
constexpr uint8_t P_IBTREE = 3, P_LBTREE = 5, P_OVERFLOW = 7, P_BTREEMETA = 9;
constexpr uint8_t B_KEYDATA = 1, B_DUPLICATE = 2, B_OVERFLOW = 3, B_DELETE = 0x80;
constexpr uint32_t BTM_SUBDB = 0x20;
constexpr size_t PAGE_HDR = 26;
constexpr int MAX_DEPTH = 64;

[[noreturn]] void fail(const std::string& what) { throw std::runtime_error("wallet.dat (Berkeley DB): " + what); }

class File {
public:
    explicit File(std::string data) : data_(std::move(data)) {
        if (data_.size() < 512) fail("file too short");
        uint32_t m;
        std::memcpy(&m, data_.data() + 12, 4);
        if (m == BTREE_MAGIC) {
            swap_ = false;
        } else if (__builtin_bswap32(m) == BTREE_MAGIC) {
            swap_ = true;
        } else {
            fail("not a btree file (magic)");
        }
        npages_ = 1;  // page 0 (the meta page) is readable while the page size is checked
        pagesize_ = u32at(0, 20);
        if (pagesize_ < 512 || pagesize_ > 65536 || (pagesize_ & (pagesize_ - 1))) fail("bad page size");
        const uint32_t version = u32at(0, 16);
        if (version < 8 || version > 10) fail("unsupported btree version " + std::to_string(version));
        if (u8at(0, 24) != 0) fail("encrypted database files are not supported");
        inp_ = PAGE_HDR + ((u8at(0, 26) & 1) ? 6 : 0);  // PG_CHKSUM area of checksummed files
        npages_ = data_.size() / pagesize_;
    }

    const uint8_t* page(uint32_t pgno) const {
        if (pgno >= npages_) fail("page " + std::to_string(pgno) + " past the end of the file");
        return reinterpret_cast<const uint8_t*>(data_.data()) + size_t(pgno) * pagesize_;
    }
    uint8_t u8at(uint32_t pgno, size_t off) const { return page(pgno)[off]; }
    uint16_t u16(const uint8_t* p) const {
        uint16_t v;
        std::memcpy(&v, p, 2);
        return swap_ ? __builtin_bswap16(v) : v;
    }
    uint32_t u32(const uint8_t* p) const {
        uint32_t v;
        std::memcpy(&v, p, 4);
        return swap_ ? __builtin_bswap32(v) : v;
    }
    uint32_t u32at(uint32_t pgno, size_t off) const { return u32(page(pgno) + off); }

    // Root page of the btree whose meta page is `meta`.
    uint32_t root_of(uint32_t meta) const {
        const uint8_t* p = page(meta);
        if (p[25] != P_BTREEMETA || u32(p + 12) != BTREE_MAGIC) fail("page " + std::to_string(meta) + " is not a btree meta page");
        return u32(p + 88);
    }
    bool has_subdbs() const { return (u32at(0, 48) & BTM_SUBDB) != 0; }

    // Offset of item `i` on page `p`, checked to lie inside the page.
    size_t item(const uint8_t* p, uint32_t i, size_t need) const {
        const size_t at = inp_ + 2 * size_t(i);
        if (at + 2 > pagesize_) fail("item index past the page");
        const size_t off = u16(p + at);
        if (off < inp_ || off + need > pagesize_) fail("item offset past the page");
        return off;
    }

    // Bytes of leaf item `i` of page `p` (inline or in an overflow chain); false if deleted.
    bool read_item(const uint8_t* p, uint32_t i, std::string& out) const {
        const size_t off = item(p, i, 3);
        const uint8_t type = p[off + 2];
        if (type & B_DELETE) return false;
        switch (type & 0x7F) {
        case B_KEYDATA: {
            const size_t len = u16(p + off);
            if (off + 3 + len > pagesize_) fail("key/data item past the page");
            out.assign(reinterpret_cast<const char*>(p + off + 3), len);
            return true;
        }
        case B_OVERFLOW: {
            item(p, i, 12);
            uint32_t next = u32(p + off + 4);
            const uint32_t total = u32(p + off + 8);
            // the chain has at most npages_ pages of payload: a length beyond that is damage, and
            // must not reserve gigabytes before the first page is checked
            if (uint64_t(total) > uint64_t(npages_) * pagesize_) fail("overflow item longer than the file");
            out.clear();
            out.reserve(total);
            for (size_t hops = 0; out.size() < total; ++hops) {
                if (hops > npages_ || next == 0) fail("broken overflow chain");
                const uint8_t* op = page(next);
                if (op[25] != P_OVERFLOW) fail("overflow item points at a non-overflow page");
                const size_t len = u16(op + 22);  // OV_LEN: hf_offset holds the payload length
                if (inp_ + len > pagesize_ || out.size() + len > total) fail("overflow page length");
                out.append(reinterpret_cast<const char*>(op + inp_), len);
                next = u32(op + 16);
            }
            return true;
        }
        case B_DUPLICATE:
            fail("off-page duplicate trees are not supported");
        default:
            fail("unknown item type " + std::to_string(type));
        }
    }

    void walk(uint32_t pgno, int depth, Records& out, std::vector<bool>& seen) const {
        if (depth > MAX_DEPTH) fail("btree deeper than " + std::to_string(MAX_DEPTH));
        const uint8_t* p = page(pgno);
        if (seen[pgno]) fail("page " + std::to_string(pgno) + " reached twice (a cycle in the tree)");
        seen[pgno] = true;
        const uint32_t entries = u16(p + 20);
        switch (p[25]) {
        case P_IBTREE:
            for (uint32_t i = 0; i < entries; ++i) {
                const size_t off = item(p, i, 12);
                walk(u32(p + off + 4), depth + 1, out, seen);
            }
            break;
        case P_LBTREE: {
            if (entries & 1) fail("leaf page with an odd item count");
            std::string k, v;
            for (uint32_t i = 0; i < entries; i += 2) {
                const bool kl = read_item(p, i, k);
                const bool vl = read_item(p, i + 1, v);
                if (kl && vl) out.emplace_back(k, v);
            }
            break;
        }
        default:
            fail("unexpected page type " + std::to_string(p[25]) + " in the btree");
        }
    }

    Records tree(uint32_t meta) const {
        Records out;
        std::vector<bool> seen(npages_, false);
        walk(root_of(meta), 0, out, seen);
        return out;
    }

    // Meta page of sub-database `name` (its master-database record, network byte order).
    uint32_t subdb_meta(const std::string& name) const {
        for (const auto& [k, v] : tree(0)) {
            if (k != name) continue;
            if (v.size() != 4) fail("bad sub-database record");
            uint32_t raw;
            std::memcpy(&raw, v.data(), 4);
            for (uint32_t cand : {__builtin_bswap32(raw), raw}) {  // network order; host order accepted
                if (cand > 0 && cand < npages_) {
                    const uint8_t* p = page(cand);
                    if (p[25] == P_BTREEMETA && u32(p + 12) == BTREE_MAGIC) return cand;
                }
            }
            fail("sub-database \"" + name + "\" points at no meta page");
        }
        fail("no sub-database \"" + name + "\"");
    }

private:
    std::string data_;
    uint32_t pagesize_ = 0;
    size_t inp_ = PAGE_HDR, npages_ = 0;
    bool swap_ = false;
};

std::string slurp(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) fail("cannot open " + path);
    return std::string(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
}

// ------------------------------------------------------------------------------ writer
constexpr uint32_t BTREE_VERSION = 9;  // Berkeley DB 4.8 .. 5.3
constexpr uint8_t LEAFLEVEL = 1;

struct Writer {
    uint32_t ps;
    std::vector<std::string> pages;  // page images, index = pgno

    explicit Writer(uint32_t pagesize) : ps(pagesize) {}

    static void put16(std::string& p, size_t off, uint16_t v) { std::memcpy(&p[off], &v, 2); }
    static void put32(std::string& p, size_t off, uint32_t v) { std::memcpy(&p[off], &v, 4); }

    uint32_t alloc(uint8_t type, uint8_t level) {
        const uint32_t pgno = uint32_t(pages.size());
        std::string p(ps, '\0');
        put32(p, 0, 0);
        put32(p, 4, 1);  // LSN {0, 1}: not logged
        put32(p, 8, pgno);
        put16(p, 22, uint16_t(ps));  // hf_offset: no items yet
        p[24] = char(level);
        p[25] = char(type);
        pages.push_back(std::move(p));
        return pgno;
    }

    // Bytes an item takes on a page (4-byte aligned) plus its index slot.
    static size_t need(size_t item_bytes) { return ((item_bytes + 3) & ~size_t(3)) + 2; }
    size_t free_bytes(uint32_t pgno) const {
        const std::string& p = pages[pgno];
        uint16_t n, hf;
        std::memcpy(&n, &p[20], 2);
        std::memcpy(&hf, &p[22], 2);
        return size_t(hf) - (PAGE_HDR + 2 * size_t(n));
    }
    // Appends an item image (below the previous ones, index slot after the previous slots).
    void add_item(uint32_t pgno, const std::string& item) {
        std::string& p = pages[pgno];
        uint16_t n, hf;
        std::memcpy(&n, &p[20], 2);
        std::memcpy(&hf, &p[22], 2);
        const size_t sz = (item.size() + 3) & ~size_t(3);
        if (sz + 2 > free_bytes(pgno)) throw std::logic_error("bdb writer: item does not fit");
        const uint16_t off = uint16_t(hf - sz);
        std::memcpy(&p[off], item.data(), item.size());
        put16(p, PAGE_HDR + 2 * size_t(n), off);
        put16(p, 20, uint16_t(n + 1));
        put16(p, 22, off);
    }
    // A BOVERFLOW item pointing at a fresh chain of overflow pages holding `data`.
    std::string overflow(const std::string& data) {
        const size_t cap = ps - PAGE_HDR;
        uint32_t first = 0, prev = 0;
        for (size_t at = 0; at < data.size(); at += cap) {
            const size_t len = std::min(cap, data.size() - at);
            const uint32_t pg = alloc(P_OVERFLOW, 0);
            std::string& p = pages[pg];
            put16(p, 20, 1);  // reference count
            put16(p, 22, uint16_t(len));  // OV_LEN: payload bytes on this page
            put32(p, 12, prev);
            std::memcpy(&p[PAGE_HDR], data.data() + at, len);
            if (prev) put32(pages[prev], 16, pg);
            if (!first) first = pg;
            prev = pg;
        }
        std::string it(12, '\0');
        it[2] = char(B_OVERFLOW);
        put32(it, 4, first);
        put32(it, 8, uint32_t(data.size()));
        return it;
    }
    static std::string keydata(const std::string& data) {
        std::string it(3, '\0');
        put16(it, 0, uint16_t(data.size()));
        it[2] = char(B_KEYDATA);
        return it + data;
    }
    void meta(uint32_t pgno, uint32_t root, uint32_t last, uint32_t flags, const std::string& uid) {
        std::string& p = pages[pgno];
        std::fill(p.begin() + 12, p.end(), '\0');  // the meta layout reuses the page-header fields
        put32(p, 12, BTREE_MAGIC);
        put32(p, 16, BTREE_VERSION);
        put32(p, 20, ps);
        p[25] = char(P_BTREEMETA);
        put32(p, 32, last);
        put32(p, 48, flags);
        std::memcpy(&p[52], uid.data(), 20);
        put32(p, 76, 2);  // minkey
        put32(p, 88, root);
    }

    // The btree of sorted `recs`: returns its root page.
    uint32_t tree(const Records& recs) {
        // items larger than the overflow size go to overflow pages (B_MINKEY_TO_OVFLSIZE, minkey 2)
        const size_t ovfl = (ps - PAGE_HDR) / 4 - 8;
        std::vector<std::pair<uint32_t, std::string>> level;  // (page, first key) of this level
        uint32_t leaf = alloc(P_LBTREE, LEAFLEVEL);
        level.emplace_back(leaf, recs.empty() ? std::string() : recs[0].first);
        for (const auto& [k, v] : recs) {
            const std::string ki = k.size() > ovfl ? overflow(k) : keydata(k);
            const std::string vi = v.size() > ovfl ? overflow(v) : keydata(v);
            if (need(ki.size()) + need(vi.size()) > free_bytes(leaf)) {
                const uint32_t next = alloc(P_LBTREE, LEAFLEVEL);
                put32(pages[leaf], 16, next);  // leaf siblings are linked
                put32(pages[next], 12, leaf);
                leaf = next;
                level.emplace_back(leaf, k);
            }
            add_item(leaf, ki);
            add_item(leaf, vi);
        }
        // internal levels until one page holds the level
        for (uint8_t lv = LEAFLEVEL + 1; level.size() > 1; ++lv) {
            std::vector<std::pair<uint32_t, std::string>> up;
            uint32_t pg = alloc(P_IBTREE, lv);
            up.emplace_back(pg, level[0].second);
            for (size_t i = 0; i < level.size(); ++i) {
                // BINTERNAL: len, type, unused, child pgno, nrecs, key (empty on a page's first entry)
                std::string key = pages[pg][20] == 0 && pages[pg][21] == 0 ? std::string() : level[i].second;
                auto item = [&](const std::string& kk) {
                    std::string it(12, '\0');
                    put16(it, 0, uint16_t(kk.size()));
                    it[2] = char(B_KEYDATA);
                    put32(it, 4, level[i].first);
                    return it + kk;
                };
                if (key.size() > ovfl) throw std::invalid_argument("bdb writer: key longer than the overflow size");
                if (need(item(key).size()) > free_bytes(pg)) {
                    pg = alloc(P_IBTREE, lv);
                    up.emplace_back(pg, level[i].second);
                    key.clear();
                }
                add_item(pg, item(key));
            }
            level.swap(up);
        }
        return level[0].first;
    }
};

}  // namespace

std::string write_btree_bytes(Records records, const std::string& subdb, uint32_t pagesize, const std::string& uid_in) {
    if (pagesize < 512 || pagesize > 65536 || (pagesize & (pagesize - 1))) throw std::invalid_argument("bad page size");
    if (subdb.empty()) throw std::invalid_argument("bdb writer: a sub-database name is required");
    // __bam_defcmp: bytewise, a prefix sorts first
    std::sort(records.begin(), records.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (size_t i = 1; i < records.size(); ++i)
        if (records[i].first == records[i - 1].first) throw std::invalid_argument("bdb writer: duplicate key");
    std::string uid = uid_in;
    if (uid.size() != 20) {
        std::random_device rd;
        uid.assign(20, '\0');
        for (auto& c : uid) c = char(rd());
    }
    Writer w(pagesize);
    w.alloc(P_BTREEMETA, 0);                  // 0: master meta
    const uint32_t mleaf = w.alloc(P_LBTREE, LEAFLEVEL);  // 1: master root leaf
    w.alloc(P_BTREEMETA, 0);                  // 2: the sub-database's meta
    const uint32_t root = w.tree(records);
    std::string pg(4, '\0');
    const uint32_t be = __builtin_bswap32(2u);  // network byte order (__db_master_update)
    std::memcpy(&pg[0], &be, 4);
    w.add_item(mleaf, Writer::keydata(subdb));
    w.add_item(mleaf, Writer::keydata(pg));
    const uint32_t last = uint32_t(w.pages.size() - 1);
    w.meta(0, mleaf, last, BTM_SUBDB, uid);
    w.meta(2, root, 2, BTM_SUBDB, uid);
    std::string out;
    out.reserve(w.pages.size() * size_t(pagesize));
    for (const auto& p : w.pages) out += p;
    return out;
}

void write_btree(const std::string& path, Records records, const std::string& subdb, uint32_t pagesize) {
    const std::string data = write_btree_bytes(std::move(records), subdb, pagesize);
    const std::string tmp = path + ".tmp";
    // written in full and synced before it takes the name: a crash leaves the old file or the new one
    std::FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + tmp);
    const bool ok = std::fwrite(data.data(), 1, data.size(), f) == data.size() && std::fflush(f) == 0 &&
                    ::fsync(::fileno(f)) == 0;
    std::fclose(f);
    if (!ok) {
        std::remove(tmp.c_str());
        throw std::runtime_error("short write to " + tmp);
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("cannot rename " + tmp);
}

Records read_btree_bytes(std::string data, const std::string& subdb) {
    File f(std::move(data));
    if (subdb.empty()) return f.tree(0);
    if (!f.has_subdbs()) fail("the file has no sub-databases");
    return f.tree(f.subdb_meta(subdb));
}

Records read_btree(const std::string& path, const std::string& subdb) { return read_btree_bytes(slurp(path), subdb); }

std::vector<std::string> databases(const std::string& path) {
    File f(slurp(path));
    std::vector<std::string> names;
    if (!f.has_subdbs()) return names;
    for (const auto& kv : f.tree(0)) names.push_back(kv.first);
    return names;
}

}  // namespace bdb
}  // namespace nodexa
