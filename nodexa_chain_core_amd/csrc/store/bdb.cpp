// Read-only Berkeley DB btree reader (see bdb.hpp for the page format it walks).
#include "bdb.hpp"

#include <cstdint>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <utility>

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

}  // namespace

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
