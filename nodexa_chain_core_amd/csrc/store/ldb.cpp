// LevelDB-format store (see ldb.hpp for the file layout and what is engine-specific).
//
// Format parity, by piece (reference sources read for behaviour: src/leveldb/db/log_format.h,
// table/format.h, table/block_builder.cc, table/filter_block.cc, util/bloom.cc, util/hash.cc,
// db/version_edit.cc, db/dbformat.h): CRC32C with the 0xa282ead8 mask, little-endian fixed
// ints and base-128 varints, internal keys = user key + (sequence << 8 | type), bytewise user-key
// order with newer sequences first, 2 KiB filter ranges (base lg 11), the double-hashing bloom
// filter keyed by the Murmur-style Hash(seed 0xbc9f1d34), magic 0xdb4775248b80fb57.
#include "ldb.hpp"

#include <dirent.h>
#include <fcntl.h>
#include <nmmintrin.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <queue>
#include <set>
#include <stdexcept>

namespace nodexa {
namespace ldb {

namespace {

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;
constexpr uint32_t kLogBlock = 32768;
constexpr uint32_t kLogHeader = 7;
constexpr uint64_t kMaxSeq = (1ull << 56) - 1;
constexpr int kFilterBaseLg = 11;
constexpr int kLevels = 7;
const char* kFilterName = "filter.leveldb.BuiltinBloomFilter2";
const char* kComparator = "leveldb.BytewiseComparator";

[[noreturn]] void fail(const std::string& what) { throw std::runtime_error("ldb: " + what); }

// ---------------------------------------------------------------- coding
void put_fixed32(std::string* d, uint32_t v) {
    char b[4];
    std::memcpy(b, &v, 4);
    d->append(b, 4);
}
void put_fixed64(std::string* d, uint64_t v) {
    char b[8];
    std::memcpy(b, &v, 8);
    d->append(b, 8);
}
uint32_t get_fixed32(const char* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}
uint64_t get_fixed64(const char* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
}
void put_varint(std::string* d, uint64_t v) {
    while (v >= 0x80) {
        d->push_back(char(v | 0x80));
        v >>= 7;
    }
    d->push_back(char(v));
}
bool get_varint(const char*& p, const char* end, uint64_t* v) {
    uint64_t r = 0;
    for (int shift = 0; shift <= 63 && p < end; shift += 7) {
        const uint8_t b = uint8_t(*p++);
        r |= uint64_t(b & 0x7f) << shift;
        if (!(b & 0x80)) {
            *v = r;
            return true;
        }
    }
    return false;
}
void put_lenpref(std::string* d, const std::string& s) {
    put_varint(d, s.size());
    d->append(s);
}
bool get_lenpref(const char*& p, const char* end, std::string* s) {
    uint64_t n;
    if (!get_varint(p, end, &n) || uint64_t(end - p) < n) return false;
    s->assign(p, size_t(n));
    p += n;
    return true;
}

// ---------------------------------------------------------------- internal keys
std::string ikey(const std::string& user, uint64_t seq, bool value) {
    std::string k = user;
    put_fixed64(&k, (seq << 8) | (value ? 1u : 0u));
    return k;
}
inline int ucmp(const char* a, size_t na, const char* b, size_t nb) {
    const int r = std::memcmp(a, b, std::min(na, nb));
    if (r) return r;
    return na < nb ? -1 : (na > nb ? 1 : 0);
}
// user key ascending, then (sequence, type) descending
int icmp(const std::string& a, const std::string& b) {
    const int r = ucmp(a.data(), a.size() - 8, b.data(), b.size() - 8);
    if (r) return r;
    const uint64_t ta = get_fixed64(a.data() + a.size() - 8), tb = get_fixed64(b.data() + b.size() - 8);
    return ta > tb ? -1 : (ta < tb ? 1 : 0);
}
std::string user_of(const std::string& ik) { return ik.substr(0, ik.size() - 8); }
bool is_value(const std::string& ik) { return (uint8_t(ik[ik.size() - 8])) == 1; }

// ---------------------------------------------------------------- files
std::string fname(const std::string& dir, uint64_t n, const char* ext) {
    char b[32];
    std::snprintf(b, sizeof b, "/%06llu.%s", (unsigned long long)n, ext);
    return dir + b;
}
std::string manifest_name(uint64_t n) {
    char b[32];
    std::snprintf(b, sizeof b, "MANIFEST-%06llu", (unsigned long long)n);
    return b;
}
bool read_file(const std::string& path, std::string* out) {
    const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return false;
    out->clear();
    char buf[1 << 16];
    for (;;) {
        const ssize_t r = ::read(fd, buf, sizeof buf);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) break;
        out->append(buf, size_t(r));
    }
    ::close(fd);
    return true;
}
void write_all(int fd, const char* p, size_t n) {
    while (n) {
        const ssize_t r = ::write(fd, p, n);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) fail(std::string("write: ") + std::strerror(errno));
        p += r;
        n -= size_t(r);
    }
}
void sync_dir(const std::string& dir) {
    const int fd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
    if (fd >= 0) {
        ::fsync(fd);
        ::close(fd);
    }
}
std::vector<std::string> list_dir(const std::string& dir) {
    std::vector<std::string> out;
    DIR* d = ::opendir(dir.c_str());
    if (!d) return out;
    while (dirent* e = ::readdir(d)) out.emplace_back(e->d_name);
    ::closedir(d);
    return out;
}
// number and kind ('l' log, 't' table, 'm' manifest, 'x' temp) of a store file name
bool parse_name(const std::string& n, uint64_t* num, char* kind) {
    auto digits = [&](const std::string& s, uint64_t* v) {
        if (s.empty() || s.size() > 19) return false;
        uint64_t r = 0;
        for (char c : s) {
            if (c < '0' || c > '9') return false;
            r = r * 10 + uint64_t(c - '0');
        }
        *v = r;
        return true;
    };
    if (n.rfind("MANIFEST-", 0) == 0) {
        *kind = 'm';
        return digits(n.substr(9), num);
    }
    const size_t dot = n.find('.');
    if (dot == std::string::npos || !digits(n.substr(0, dot), num)) return false;
    const std::string ext = n.substr(dot + 1);
    if (ext == "log") *kind = 'l';
    else if (ext == "ldb" || ext == "sst") *kind = 't';
    else if (ext == "dbtmp") *kind = 'x';
    else return false;
    return true;
}

// ---------------------------------------------------------------- log records
void log_append(int fd, uint32_t* block_off, const std::string& payload) {
    const char* p = payload.data();
    size_t left = payload.size();
    bool begin = true;
    std::string out;
    do {
        const uint32_t leftover = kLogBlock - *block_off;
        if (leftover < kLogHeader) {
            out.append(leftover, '\0');
            *block_off = 0;
        }
        const size_t avail = kLogBlock - *block_off - kLogHeader;
        const size_t frag = std::min(left, avail);
        const bool end = frag == left;
        const uint8_t type = begin && end ? 1 : begin ? 2 : end ? 4 : 3;
        const uint32_t crc = crc_mask(crc32c(p, frag, crc32c(&type, 1)));
        put_fixed32(&out, crc);
        out.push_back(char(frag & 0xff));
        out.push_back(char(frag >> 8));
        out.push_back(char(type));
        out.append(p, frag);
        *block_off += uint32_t(kLogHeader + frag);
        p += frag;
        left -= frag;
        begin = false;
    } while (left > 0);
    write_all(fd, out.data(), out.size());
}

// Complete records of a log file in order. A torn or corrupt record ends its block's records
// (and any fragmented record it belonged to), as the reference's reader reports and skips them.
std::vector<std::string> log_records(const std::string& data) {
    std::vector<std::string> out;
    std::string scratch;
    bool in_frag = false;
    size_t off = 0;
    while (off < data.size()) {
        const size_t block_left = kLogBlock - off % kLogBlock;
        if (block_left < kLogHeader || off + kLogHeader > data.size()) {
            off += block_left;
            continue;
        }
        const char* h = data.data() + off;
        const uint32_t len = uint8_t(h[4]) | (uint32_t(uint8_t(h[5])) << 8);
        const uint8_t type = uint8_t(h[6]);
        if (type == 0 && len == 0) {  // zero padding
            off += block_left;
            continue;
        }
        if (kLogHeader + len > block_left || off + kLogHeader + len > data.size()) break;  // torn tail
        const uint32_t stored = get_fixed32(h);
        const uint32_t rot = stored - 0xa282ead8u;
        const uint32_t crc = (rot >> 17) | (rot << 15);
        if (crc != crc32c(h + kLogHeader, len, crc32c(&type, 1))) {
            in_frag = false;
            off += block_left;  // skip the rest of the damaged block
            continue;
        }
        const std::string frag(h + kLogHeader, len);
        switch (type) {
            case 1: out.push_back(frag); in_frag = false; break;
            case 2: scratch = frag; in_frag = true; break;
            case 3: if (in_frag) scratch += frag; break;
            case 4:
                if (in_frag) out.push_back(scratch + frag);
                in_frag = false;
                break;
            default: break;
        }
        off += kLogHeader + len;
    }
    return out;
}

// ---------------------------------------------------------------- blocks
struct Handle {
    uint64_t offset = 0, size = 0;
    std::string encode() const {
        std::string s;
        put_varint(&s, offset);
        put_varint(&s, size);
        return s;
    }
    bool decode(const char*& p, const char* end) { return get_varint(p, end, &offset) && get_varint(p, end, &size); }
};

class BlockBuilder {
public:
    explicit BlockBuilder(int interval) : interval_(interval) { restarts_.push_back(0); }
    void add(const std::string& key, const std::string& value) {
        size_t shared = 0;
        if (counter_ < interval_) {
            const size_t lim = std::min(last_.size(), key.size());
            while (shared < lim && last_[shared] == key[shared]) ++shared;
        } else {
            restarts_.push_back(uint32_t(buf_.size()));
            counter_ = 0;
        }
        put_varint(&buf_, shared);
        put_varint(&buf_, key.size() - shared);
        put_varint(&buf_, value.size());
        buf_.append(key, shared, std::string::npos);
        buf_.append(value);
        last_ = key;
        ++counter_;
        ++entries_;
    }
    size_t estimate() const { return buf_.size() + restarts_.size() * 4 + 4; }
    bool empty() const { return entries_ == 0; }
    std::string finish() {
        std::string out = buf_;
        for (uint32_t r : restarts_) put_fixed32(&out, r);
        put_fixed32(&out, uint32_t(restarts_.size()));
        return out;
    }
    void reset() {
        buf_.clear();
        restarts_.assign(1, 0);
        counter_ = 0;
        entries_ = 0;
        last_.clear();
    }

private:
    int interval_;
    std::string buf_, last_;
    std::vector<uint32_t> restarts_;
    int counter_ = 0;
    size_t entries_ = 0;
};

bool decode_block(const std::string& b, std::vector<std::pair<std::string, std::string>>* out) {
    out->clear();
    if (b.size() < 4) return false;
    const uint32_t nr = get_fixed32(b.data() + b.size() - 4);
    if (uint64_t(nr) * 4 + 4 > b.size()) return false;
    const char* p = b.data();
    const char* end = b.data() + b.size() - 4 - size_t(nr) * 4;
    std::string key;
    while (p < end) {
        uint64_t shared, non_shared, vlen;
        if (!get_varint(p, end, &shared) || !get_varint(p, end, &non_shared) || !get_varint(p, end, &vlen)) return false;
        if (shared > key.size() || uint64_t(end - p) < non_shared + vlen) return false;
        key.resize(size_t(shared));
        key.append(p, size_t(non_shared));
        p += non_shared;
        out->emplace_back(key, std::string(p, size_t(vlen)));
        p += vlen;
    }
    return true;
}

// ---------------------------------------------------------------- bloom filter
void bloom_create(const std::vector<std::string>& keys, int bits_per_key, std::string* dst) {
    size_t bits = keys.size() * size_t(bits_per_key);
    if (bits < 64) bits = 64;
    const size_t bytes = (bits + 7) / 8;
    bits = bytes * 8;
    size_t k = size_t(bits_per_key * 0.69);
    k = std::max<size_t>(1, std::min<size_t>(30, k));
    const size_t init = dst->size();
    dst->resize(init + bytes, '\0');
    dst->push_back(char(k));
    char* array = &(*dst)[init];
    for (const std::string& key : keys) {
        uint32_t h = bloom_hash(key);
        const uint32_t delta = (h >> 17) | (h << 15);
        for (size_t j = 0; j < k; ++j) {
            const uint32_t pos = h % uint32_t(bits);
            array[pos / 8] |= char(1 << (pos % 8));
            h += delta;
        }
    }
}
bool bloom_may_match(const std::string& key, const char* f, size_t len) {
    if (len < 2) return false;
    const size_t k = uint8_t(f[len - 1]);
    if (k > 30) return true;  // reserved for other encodings
    const uint32_t bits = uint32_t((len - 1) * 8);
    uint32_t h = bloom_hash(key);
    const uint32_t delta = (h >> 17) | (h << 15);
    for (size_t j = 0; j < k; ++j) {
        const uint32_t pos = h % bits;
        if (!(f[pos / 8] & (1 << (pos % 8)))) return false;
        h += delta;
    }
    return true;
}

// ---------------------------------------------------------------- table writer
class TableBuilder {
public:
    TableBuilder(const std::string& path, const Options& opt)
        : opt_(opt), data_(opt.block_restart_interval), index_(1) {
        fd_ = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
        if (fd_ < 0) fail("create " + path + ": " + std::strerror(errno));
    }
    ~TableBuilder() {
        if (fd_ >= 0) ::close(fd_);
    }
    void add(const std::string& ik, const std::string& value) {
        if (pending_index_) {
            index_.add(last_key_, pending_.encode());
            pending_index_ = false;
        }
        if (opt_.bloom_bits_per_key > 0) filter_keys_.push_back(user_of(ik));
        if (entries_ == 0) smallest_ = ik;
        last_key_ = ik;
        data_.add(ik, value);
        ++entries_;
        if (data_.estimate() >= opt_.block_size) flush();
    }
    uint64_t file_size() const { return offset_ + data_.estimate(); }
    uint64_t entries() const { return entries_; }
    FileMeta finish(uint64_t number) {
        flush();
        Handle filter_h, meta_h, index_h;
        BlockBuilder meta(opt_.block_restart_interval);
        if (opt_.bloom_bits_per_key > 0) {
            if (!filter_keys_.empty()) gen_filter();
            const uint32_t array_off = uint32_t(filter_.size());
            for (uint32_t o : filter_offsets_) put_fixed32(&filter_, o);
            put_fixed32(&filter_, array_off);
            filter_.push_back(char(kFilterBaseLg));
            filter_h = write_raw(filter_);
            meta.add(kFilterName, filter_h.encode());
        }
        meta_h = write_raw(meta.finish());
        if (pending_index_) {
            index_.add(last_key_, pending_.encode());
            pending_index_ = false;
        }
        index_h = write_raw(index_.finish());
        std::string footer = meta_h.encode() + index_h.encode();
        footer.resize(40, '\0');
        put_fixed64(&footer, kTableMagic);
        write_all(fd_, footer.data(), footer.size());
        offset_ += footer.size();
        if (::fsync(fd_) != 0) fail("fsync table");
        ::close(fd_);
        fd_ = -1;
        FileMeta m;
        m.number = number;
        m.size = offset_;
        m.smallest = smallest_;
        m.largest = last_key_;
        return m;
    }

private:
    void flush() {
        if (data_.empty()) return;
        pending_ = write_raw(data_.finish());
        data_.reset();
        pending_index_ = true;
        // the next data block starts at offset_: its keys go to the filter of that 2 KiB range
        const uint64_t idx = offset_ >> kFilterBaseLg;
        if (opt_.bloom_bits_per_key > 0)
            while (idx > filter_offsets_.size()) gen_filter();
    }
    void gen_filter() {
        filter_offsets_.push_back(uint32_t(filter_.size()));
        if (filter_keys_.empty()) return;
        bloom_create(filter_keys_, opt_.bloom_bits_per_key, &filter_);
        filter_keys_.clear();
    }
    Handle write_raw(const std::string& contents) {
        Handle h{offset_, contents.size()};
        const uint8_t type = 0;  // no compression (CDBWrapper sets kNoCompression)
        std::string trailer(1, char(type));
        put_fixed32(&trailer, crc_mask(crc32c(&type, 1, crc32c(contents.data(), contents.size()))));
        write_all(fd_, contents.data(), contents.size());
        write_all(fd_, trailer.data(), trailer.size());
        offset_ += contents.size() + trailer.size();
        return h;
    }

    Options opt_;
    int fd_ = -1;
    uint64_t offset_ = 0, entries_ = 0;
    BlockBuilder data_, index_;
    bool pending_index_ = false;
    Handle pending_;
    std::string last_key_, smallest_;
    std::vector<std::string> filter_keys_;
    std::string filter_;
    std::vector<uint32_t> filter_offsets_;
};

}  // namespace

// ---------------------------------------------------------------- table reader
class Table {
public:
    Table(const std::string& path, uint64_t size) : path_(path) {
        fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
        if (fd_ < 0) fail("open table " + path + ": " + std::strerror(errno));
        struct stat st;
        if (::fstat(fd_, &st) != 0) fail("stat " + path);
        size_ = uint64_t(st.st_size);
        (void)size;
        if (size_ < 48) fail("table too short: " + path);
        std::string footer = pread_str(size_ - 48, 48);
        if (get_fixed64(footer.data() + 40) != kTableMagic) fail("bad table magic: " + path);
        const char* p = footer.data();
        Handle meta_h, index_h;
        if (!meta_h.decode(p, footer.data() + 40) || !index_h.decode(p, footer.data() + 40)) fail("bad footer: " + path);
        std::vector<std::pair<std::string, std::string>> entries;
        if (!decode_block(read_block(index_h), &entries)) fail("bad index block: " + path);
        for (auto& e : entries) {
            const char* q = e.second.data();
            Handle h;
            if (!h.decode(q, e.second.data() + e.second.size())) fail("bad index entry: " + path);
            index_.emplace_back(std::move(e.first), h);
        }
        if (!decode_block(read_block(meta_h), &entries)) fail("bad metaindex block: " + path);
        for (auto& e : entries) {
            if (e.first != kFilterName) continue;
            const char* q = e.second.data();
            Handle h;
            if (!h.decode(q, e.second.data() + e.second.size())) break;
            filter_ = read_block(h);
            if (filter_.size() >= 5) {
                base_lg_ = uint8_t(filter_[filter_.size() - 1]);
                array_off_ = get_fixed32(filter_.data() + filter_.size() - 5);
                if (array_off_ <= filter_.size() - 5) num_filters_ = (filter_.size() - 5 - array_off_) / 4;
            }
        }
    }
    ~Table() {
        if (fd_ >= 0) ::close(fd_);
    }
    // Newest entry for `user` in this table: 0 absent, 1 value, 2 deletion.
    int get(const std::string& user, std::string* value) {
        const std::string seek = ikey(user, kMaxSeq, true);
        size_t lo = 0, hi = index_.size();
        while (lo < hi) {
            const size_t mid = (lo + hi) / 2;
            if (icmp(index_[mid].first, seek) < 0) lo = mid + 1;
            else hi = mid;
        }
        if (lo == index_.size()) return 0;
        const Handle& h = index_[lo].second;
        if (!may_match(h.offset, user)) return 0;
        std::vector<std::pair<std::string, std::string>> entries;
        if (!decode_block(read_block(h), &entries)) fail("bad data block: " + path_);
        for (auto& e : entries) {
            if (e.first.size() < 8 || icmp(e.first, seek) < 0) continue;
            if (ucmp(e.first.data(), e.first.size() - 8, user.data(), user.size()) != 0) return 0;
            if (!is_value(e.first)) return 2;
            *value = std::move(e.second);
            return 1;
        }
        return 0;
    }
    size_t blocks() const { return index_.size(); }
    // entries of data block i (in internal-key order)
    void block(size_t i, std::vector<std::pair<std::string, std::string>>* out) {
        if (!decode_block(read_block(index_[i].second), out)) fail("bad data block: " + path_);
    }
    // first data block that can hold internal keys >= `seek`
    size_t lower_block(const std::string& seek) const {
        size_t lo = 0, hi = index_.size();
        while (lo < hi) {
            const size_t mid = (lo + hi) / 2;
            if (icmp(index_[mid].first, seek) < 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }

private:
    std::string pread_str(uint64_t off, uint64_t n) {
        std::string s(size_t(n), '\0');
        size_t got = 0;
        while (got < n) {
            const ssize_t r = ::pread(fd_, &s[got], size_t(n) - got, off_t(off + got));
            if (r < 0 && errno == EINTR) continue;
            if (r <= 0) fail("short read: " + path_);
            got += size_t(r);
        }
        return s;
    }
    std::string read_block(const Handle& h) {
        if (h.offset + h.size + 5 > size_) fail("block out of range: " + path_);
        std::string raw = pread_str(h.offset, h.size + 5);
        const uint8_t type = uint8_t(raw[size_t(h.size)]);
        const uint32_t stored = get_fixed32(raw.data() + h.size + 1);
        const uint32_t rot = stored - 0xa282ead8u;
        const uint32_t crc = (rot >> 17) | (rot << 15);
        if (crc != crc32c(raw.data(), size_t(h.size) + 1)) fail("block checksum mismatch: " + path_);
        raw.resize(size_t(h.size));
        if (type == 0) return raw;
        if (type == 1) {
            std::string out;
            if (!snappy_uncompress(raw.data(), raw.size(), &out)) fail("bad snappy block: " + path_);
            return out;
        }
        fail("unknown block compression: " + path_);
    }
    bool may_match(uint64_t block_offset, const std::string& user) const {
        if (filter_.empty()) return true;
        const uint64_t idx = block_offset >> base_lg_;
        if (idx >= num_filters_) return true;
        const uint32_t start = get_fixed32(filter_.data() + array_off_ + idx * 4);
        const uint32_t limit = get_fixed32(filter_.data() + array_off_ + idx * 4 + 4);
        if (start <= limit && limit <= array_off_) return bloom_may_match(user, filter_.data() + start, limit - start);
        if (start == limit) return false;
        return true;
    }

    std::string path_;
    int fd_ = -1;
    uint64_t size_ = 0;
    std::vector<std::pair<std::string, Handle>> index_;
    std::string filter_;
    uint32_t array_off_ = 0;
    uint64_t num_filters_ = 0;
    uint8_t base_lg_ = kFilterBaseLg;
};

namespace {

// ---------------------------------------------------------------- merge cursors
struct Cursor {
    virtual ~Cursor() = default;
    virtual bool valid() const = 0;
    virtual const std::string& key() const = 0;  // internal key
    virtual const std::string& value() const = 0;
    virtual void next() = 0;
};

class TableCursor : public Cursor {
public:
    TableCursor(std::shared_ptr<Table> t, const std::string& seek) : t_(std::move(t)) {
        blk_ = t_->lower_block(seek);
        load();
        while (valid() && icmp(key(), seek) < 0) next();
    }
    bool valid() const override { return blk_ < t_->blocks() && pos_ < entries_.size(); }
    const std::string& key() const override { return entries_[pos_].first; }
    const std::string& value() const override { return entries_[pos_].second; }
    void next() override {
        if (++pos_ >= entries_.size()) {
            ++blk_;
            load();
        }
    }

private:
    void load() {
        pos_ = 0;
        entries_.clear();
        while (blk_ < t_->blocks()) {
            t_->block(blk_, &entries_);
            if (!entries_.empty()) return;
            ++blk_;
        }
    }
    std::shared_ptr<Table> t_;
    size_t blk_ = 0, pos_ = 0;
    std::vector<std::pair<std::string, std::string>> entries_;
};

struct MemRow {
    std::string ik, value;
};
class VecCursor : public Cursor {
public:
    explicit VecCursor(std::vector<MemRow> rows) : rows_(std::move(rows)) {}
    bool valid() const override { return i_ < rows_.size(); }
    const std::string& key() const override { return rows_[i_].ik; }
    const std::string& value() const override { return rows_[i_].value; }
    void next() override { ++i_; }

private:
    std::vector<MemRow> rows_;
    size_t i_ = 0;
};

// k-way merge in internal-key order
class Merger {
public:
    explicit Merger(std::vector<std::unique_ptr<Cursor>> cs) : cs_(std::move(cs)) {
        for (size_t i = 0; i < cs_.size(); ++i)
            if (cs_[i]->valid()) heap_.push_back(i);
        std::make_heap(heap_.begin(), heap_.end(), Cmp{this});
    }
    bool valid() const { return !heap_.empty(); }
    Cursor* top() const { return cs_[heap_.front()].get(); }
    void next() {
        std::pop_heap(heap_.begin(), heap_.end(), Cmp{this});
        const size_t i = heap_.back();
        heap_.pop_back();
        cs_[i]->next();
        if (cs_[i]->valid()) {
            heap_.push_back(i);
            std::push_heap(heap_.begin(), heap_.end(), Cmp{this});
        }
    }

private:
    struct Cmp {
        const Merger* m;
        bool operator()(size_t a, size_t b) const { return icmp(m->cs_[a]->key(), m->cs_[b]->key()) > 0; }
    };
    std::vector<std::unique_ptr<Cursor>> cs_;
    std::vector<size_t> heap_;
};

}  // namespace

// ---------------------------------------------------------------- public helpers
__attribute__((target("sse4.2"))) uint32_t crc32c(const void* data, size_t n, uint32_t init) {
    const uint8_t* p = static_cast<const uint8_t*>(data);
    uint64_t c = init ^ 0xffffffffu;
    while (n >= 8) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        c = _mm_crc32_u64(c, w);
        p += 8;
        n -= 8;
    }
    uint32_t c32 = uint32_t(c);
    while (n--) c32 = _mm_crc32_u8(c32, *p++);
    return c32 ^ 0xffffffffu;
}
uint32_t crc_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }

uint32_t bloom_hash(const std::string& key) {
    const uint32_t m = 0xc6a4a793u;
    const uint8_t* p = reinterpret_cast<const uint8_t*>(key.data());
    size_t n = key.size();
    uint32_t h = 0xbc9f1d34u ^ uint32_t(n * m);
    while (n >= 4) {
        uint32_t w;
        std::memcpy(&w, p, 4);
        h += w;
        h *= m;
        h ^= (h >> 16);
        p += 4;
        n -= 4;
    }
    switch (n) {
        case 3: h += uint32_t(p[2]) << 16; [[fallthrough]];
        case 2: h += uint32_t(p[1]) << 8; [[fallthrough]];
        case 1:
            h += p[0];
            h *= m;
            h ^= (h >> 24);
            break;
        default: break;
    }
    return h;
}

bool snappy_uncompress(const char* in, size_t n, std::string* out) {
    const char* p = in;
    const char* end = in + n;
    uint64_t ulen;
    if (!get_varint(p, end, &ulen) || ulen > (1ull << 32)) return false;
    out->clear();
    out->reserve(size_t(ulen));
    while (p < end) {
        const uint8_t tag = uint8_t(*p++);
        size_t len, off;
        switch (tag & 3) {
            case 0: {
                len = (tag >> 2) + 1;
                if (len > 60) {
                    const size_t nb = len - 60;
                    if (size_t(end - p) < nb) return false;
                    len = 0;
                    for (size_t i = 0; i < nb; ++i) len |= size_t(uint8_t(p[i])) << (8 * i);
                    len += 1;
                    p += nb;
                }
                if (size_t(end - p) < len) return false;
                out->append(p, len);
                p += len;
                continue;
            }
            case 1:
                if (p >= end) return false;
                len = ((tag >> 2) & 7) + 4;
                off = (size_t(tag >> 5) << 8) | uint8_t(*p++);
                break;
            case 2:
                if (end - p < 2) return false;
                len = (tag >> 2) + 1;
                off = uint8_t(p[0]) | (size_t(uint8_t(p[1])) << 8);
                p += 2;
                break;
            default:
                if (end - p < 4) return false;
                len = (tag >> 2) + 1;
                off = get_fixed32(p);
                p += 4;
                break;
        }
        if (off == 0 || off > out->size()) return false;
        const size_t from = out->size() - off;
        for (size_t i = 0; i < len; ++i) out->push_back((*out)[from + i]);  // overlapping copies repeat
    }
    return out->size() == ulen;
}

void destroy(const std::string& dir) {
    for (const std::string& n : list_dir(dir)) {
        uint64_t num;
        char kind;
        if (parse_name(n, &num, &kind) || n == "CURRENT" || n == "LOCK" || n == "LOG" || n == "LOG.old")
            ::unlink((dir + "/" + n).c_str());
    }
    ::rmdir(dir.c_str());
}

// ---------------------------------------------------------------- DB
DB::DB(const std::string& dir, const Options& opt) : dir_(dir), opt_(opt) {}

namespace {
// Stores this process has open. fcntl locks belong to the process (a second open of the same
// store in this process would succeed, and closing either descriptor would drop the lock for
// both), so like LevelDB's PosixLockTable the process keeps its own set as well.
std::mutex g_open_mu;
std::set<std::string> g_open_dirs;

std::string canonical_dir(const std::string& dir) {
    char buf[PATH_MAX];
    return ::realpath(dir.c_str(), buf) ? std::string(buf) : dir;
}
}  // namespace

std::unique_ptr<DB> DB::open(const std::string& dir, const Options& opt) {
    std::unique_ptr<DB> db(new DB(dir, opt));
    if (opt.create_if_missing) ::mkdir(dir.c_str(), 0755);
    {
        std::lock_guard<std::mutex> g(g_open_mu);
        const std::string key = canonical_dir(dir);
        if (!g_open_dirs.insert(key).second) fail("store " + dir + " is already open in this process");
        db->open_key_ = key;
    }
    db->lock_fd_ = ::open((dir + "/LOCK").c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
    if (db->lock_fd_ < 0) fail("cannot open " + dir + "/LOCK: " + std::strerror(errno));
    struct flock fl;
    std::memset(&fl, 0, sizeof fl);
    fl.l_type = F_WRLCK;
    fl.l_whence = SEEK_SET;
    if (::fcntl(db->lock_fd_, F_SETLK, &fl) != 0) fail("store " + dir + " is in use by another process");
    std::string cur;
    const bool exists = read_file(dir + "/CURRENT", &cur);
    if (exists && opt.error_if_exists) fail(dir + " exists");
    if (!exists && !opt.create_if_missing) fail(dir + " does not exist");
    if (exists) db->recover();
    db->new_log();
    db->write_snapshot_manifest();
    db->delete_obsolete();
    return db;
}

DB::~DB() {
    try {
        close();
    } catch (...) {
    }
}

void DB::close() {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) return;
    closed_ = true;
    if (log_fd_ >= 0) {
        ::fsync(log_fd_);
        ::close(log_fd_);
    }
    if (manifest_fd_ >= 0) ::close(manifest_fd_);
    tables_.clear();
    table_used_.clear();
    if (lock_fd_ >= 0) ::close(lock_fd_);  // releases the fcntl lock
    log_fd_ = manifest_fd_ = lock_fd_ = -1;
    if (!open_key_.empty()) {
        std::lock_guard<std::mutex> og(g_open_mu);
        g_open_dirs.erase(open_key_);
        open_key_.clear();
    }
}

void DB::recover() {
    std::string cur;
    read_file(dir_ + "/CURRENT", &cur);
    while (!cur.empty() && (cur.back() == '\n' || cur.back() == '\r')) cur.pop_back();
    std::string man;
    if (cur.empty() || !read_file(dir_ + "/" + cur, &man)) fail("CURRENT names a missing manifest: " + cur);
    std::map<uint64_t, FileMeta> files[kLevels];
    uint64_t prev_log = 0;
    bool have_cmp = false;
    for (const std::string& rec : log_records(man)) {
        const char* p = rec.data();
        const char* end = p + rec.size();
        while (p < end) {
            uint64_t tag, v, lvl;
            if (!get_varint(p, end, &tag)) fail("bad manifest record");
            std::string s, s2;
            switch (tag) {
                case 1:
                    if (!get_lenpref(p, end, &s)) fail("bad comparator");
                    if (s != kComparator) fail("unsupported comparator " + s);
                    have_cmp = true;
                    break;
                case 2: if (!get_varint(p, end, &log_number_)) fail("bad log number"); break;
                case 9: if (!get_varint(p, end, &prev_log)) fail("bad prev log number"); break;
                case 3: if (!get_varint(p, end, &v)) fail("bad next file"); next_file_ = std::max(next_file_, v); break;
                case 4: if (!get_varint(p, end, &v)) fail("bad last sequence"); last_seq_ = std::max(last_seq_, v); break;
                case 5:
                    if (!get_varint(p, end, &lvl) || !get_lenpref(p, end, &s)) fail("bad compact pointer");
                    break;
                case 6:
                    if (!get_varint(p, end, &lvl) || !get_varint(p, end, &v) || lvl >= kLevels) fail("bad deleted file");
                    files[lvl].erase(v);
                    break;
                case 7: {
                    FileMeta m;
                    if (!get_varint(p, end, &lvl) || !get_varint(p, end, &m.number) || !get_varint(p, end, &m.size) ||
                        !get_lenpref(p, end, &m.smallest) || !get_lenpref(p, end, &m.largest) || lvl >= kLevels ||
                        m.smallest.size() < 8 || m.largest.size() < 8)
                        fail("bad new file");
                    files[lvl][m.number] = m;
                    break;
                }
                default: fail("unknown manifest tag " + std::to_string(tag));
            }
        }
    }
    (void)have_cmp;
    uint64_t mnum;
    char kind;
    if (parse_name(cur, &mnum, &kind)) next_file_ = std::max(next_file_, mnum + 1);
    for (int l = 0; l < kLevels; ++l) {
        levels_[l].clear();
        for (auto& kv : files[l]) levels_[l].push_back(kv.second);
        if (l > 0)
            std::sort(levels_[l].begin(), levels_[l].end(),
                      [](const FileMeta& a, const FileMeta& b) { return icmp(a.smallest, b.smallest) < 0; });
    }
    // write-ahead logs not yet folded into a table, oldest first
    std::vector<uint64_t> logs;
    for (const std::string& n : list_dir(dir_)) {
        uint64_t num;
        if (!parse_name(n, &num, &kind)) continue;
        next_file_ = std::max(next_file_, num + 1);
        if (kind == 'l' && (num >= log_number_ || num == prev_log)) logs.push_back(num);
    }
    std::sort(logs.begin(), logs.end());
    for (uint64_t n : logs) replay_log(n);
    flush_memtable_locked();
}

void DB::replay_log(uint64_t number) {
    std::string data;
    if (!read_file(fname(dir_, number, "log"), &data)) return;
    for (const std::string& rec : log_records(data)) {
        if (rec.size() < 12) continue;
        const uint64_t seq = get_fixed64(rec.data());
        const uint32_t count = get_fixed32(rec.data() + 8);
        const char* p = rec.data() + 12;
        const char* end = rec.data() + rec.size();
        for (uint32_t i = 0; i < count && p < end; ++i) {
            const uint8_t t = uint8_t(*p++);
            std::string k, v;
            if (!get_lenpref(p, end, &k)) fail("bad write batch in log");
            if (t == 1 && !get_lenpref(p, end, &v)) fail("bad write batch value in log");
            MemEntry& e = mem_[k];
            mem_bytes_ += k.size() + v.size() + 32;
            e.seq = seq + i;
            e.del = t != 1;
            e.value = std::move(v);
        }
        if (count) last_seq_ = std::max(last_seq_, seq + count - 1);
    }
}

void DB::new_log() {
    const uint64_t n = next_file_++;
    const int fd = ::open(fname(dir_, n, "log").c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) fail("create log: " + std::string(std::strerror(errno)));
    if (log_fd_ >= 0) ::close(log_fd_);
    log_fd_ = fd;
    log_number_ = n;
    log_block_off_ = 0;
}

void DB::write_snapshot_manifest() {
    const uint64_t n = next_file_++;
    const std::string name = manifest_name(n);
    const int fd = ::open((dir_ + "/" + name).c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) fail("create manifest: " + std::string(std::strerror(errno)));
    std::string e;
    put_varint(&e, 1);
    put_lenpref(&e, kComparator);
    put_varint(&e, 2);
    put_varint(&e, log_number_);
    put_varint(&e, 9);
    put_varint(&e, 0);
    put_varint(&e, 3);
    put_varint(&e, next_file_);
    put_varint(&e, 4);
    put_varint(&e, last_seq_);
    for (int l = 0; l < kLevels; ++l)
        for (const FileMeta& m : levels_[l]) {
            put_varint(&e, 7);
            put_varint(&e, uint64_t(l));
            put_varint(&e, m.number);
            put_varint(&e, m.size);
            put_lenpref(&e, m.smallest);
            put_lenpref(&e, m.largest);
        }
    uint32_t off = 0;
    log_append(fd, &off, e);
    if (::fsync(fd) != 0) fail("fsync manifest");
    char tmpn[32];
    std::snprintf(tmpn, sizeof tmpn, "/%06llu.dbtmp", (unsigned long long)n);
    const std::string tmp = dir_ + tmpn;
    const int cf = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (cf < 0) fail("create CURRENT");
    const std::string body = name + "\n";
    write_all(cf, body.data(), body.size());
    ::fsync(cf);
    ::close(cf);
    if (::rename(tmp.c_str(), (dir_ + "/CURRENT").c_str()) != 0) fail("rename CURRENT");
    sync_dir(dir_);
    if (manifest_fd_ >= 0) ::close(manifest_fd_);
    manifest_fd_ = fd;
    manifest_number_ = n;
    manifest_block_off_ = off;
}

void DB::append_edit(const std::string& edit) {
    log_append(manifest_fd_, &manifest_block_off_, edit);
    if (::fsync(manifest_fd_) != 0) fail("fsync manifest");
}

void DB::delete_obsolete() {
    std::vector<uint64_t> live;
    for (int l = 0; l < kLevels; ++l)
        for (const FileMeta& m : levels_[l]) live.push_back(m.number);
    for (const std::string& n : list_dir(dir_)) {
        uint64_t num;
        char kind;
        if (!parse_name(n, &num, &kind)) continue;
        bool keep = true;
        if (kind == 'l') keep = num >= log_number_;
        else if (kind == 'm') keep = num == manifest_number_;
        else if (kind == 't') keep = std::find(live.begin(), live.end(), num) != live.end();
        else if (kind == 'x') keep = false;
        if (!keep) {
            if (kind == 't') {
                tables_.erase(num);
                table_used_.erase(num);
            }
            ::unlink((dir_ + "/" + n).c_str());
        }
    }
}

std::shared_ptr<Table> DB::table(uint64_t number, uint64_t size) {
    const uint64_t stamp = ++table_clock_;
    auto it = tables_.find(number);
    if (it != tables_.end()) {
        table_used_[number] = stamp;
        return it->second;
    }
    // bounded like the reference's max_open_files: a full chainstate has thousands of tables, each
    // an open descriptor plus its index and filter blocks; the least recently used one is closed
    // (a scan that only runs when a table is opened past the bound)
    if (tables_.size() >= std::max<size_t>(1, opt_.max_open_files)) {
        auto victim = std::min_element(table_used_.begin(), table_used_.end(),
                                       [](const auto& a, const auto& b) { return a.second < b.second; });
        tables_.erase(victim->first);
        table_used_.erase(victim);
    }
    std::string path = fname(dir_, number, "ldb");
    struct stat st;
    if (::stat(path.c_str(), &st) != 0) path = fname(dir_, number, "sst");
    auto t = std::make_shared<Table>(path, size);
    tables_[number] = t;
    table_used_[number] = stamp;
    return t;
}

std::vector<FileMeta> DB::build_tables(int, const std::function<bool(std::string*, std::string*)>& next, bool split) {
    std::vector<FileMeta> out;
    std::unique_ptr<TableBuilder> b;
    uint64_t num = 0;
    std::string k, v;
    while (next(&k, &v)) {
        if (!b) {
            num = next_file_++;
            b.reset(new TableBuilder(fname(dir_, num, "ldb"), opt_));
        }
        b->add(k, v);
        if (split && b->file_size() >= opt_.max_file_size) {
            out.push_back(b->finish(num));
            b.reset();
        }
    }
    if (b) {
        if (b->entries()) out.push_back(b->finish(num));
        else ::unlink(fname(dir_, num, "ldb").c_str());
    }
    return out;
}

void DB::flush_memtable_locked() {
    if (mem_.empty()) return;
    auto it = mem_.begin();
    std::vector<FileMeta> files = build_tables(0, [&](std::string* k, std::string* v) {
        if (it == mem_.end()) return false;
        *k = ikey(it->first, it->second.seq, !it->second.del);
        *v = it->second.value;
        ++it;
        return true;
    }, false);
    const uint64_t old_log = log_number_;
    if (manifest_fd_ >= 0) new_log();  // (during recover the caller opens the log afterwards)
    std::string e;
    put_varint(&e, 2);
    put_varint(&e, log_number_);
    put_varint(&e, 9);
    put_varint(&e, 0);
    put_varint(&e, 3);
    put_varint(&e, next_file_);
    put_varint(&e, 4);
    put_varint(&e, last_seq_);
    for (const FileMeta& m : files) {
        put_varint(&e, 7);
        put_varint(&e, 0);
        put_varint(&e, m.number);
        put_varint(&e, m.size);
        put_lenpref(&e, m.smallest);
        put_lenpref(&e, m.largest);
        levels_[0].push_back(m);
    }
    if (manifest_fd_ >= 0) {
        append_edit(e);
        if (old_log != log_number_) ::unlink(fname(dir_, old_log, "log").c_str());
    }
    mem_.clear();
    mem_bytes_ = 0;
}

uint64_t DB::level_bytes(int level) const {
    uint64_t s = 0;
    for (const FileMeta& m : levels_[level]) s += m.size;
    return s;
}

bool DB::tombstone_needed(const std::string& user, int out_level) const {
    for (int l = out_level + 1; l < kLevels; ++l)
        for (const FileMeta& m : levels_[l]) {
            const std::string lo = user_of(m.smallest), hi = user_of(m.largest);
            if (lo <= user && user <= hi) return true;
        }
    return false;
}

void DB::compact_level(int level, bool whole) {
    std::vector<FileMeta> in0, in1;
    if (level == 0 || whole) {
        in0 = levels_[level];
    } else {
        const size_t i = compact_cursor_[level]++ % levels_[level].size();
        in0.push_back(levels_[level][i]);
    }
    if (in0.empty()) return;
    std::string lo = user_of(in0[0].smallest), hi = user_of(in0[0].largest);
    for (const FileMeta& m : in0) {
        lo = std::min(lo, user_of(m.smallest));
        hi = std::max(hi, user_of(m.largest));
    }
    const int out = level + 1;
    for (const FileMeta& m : levels_[out])
        if (!(user_of(m.largest) < lo || hi < user_of(m.smallest))) in1.push_back(m);
    std::vector<std::unique_ptr<Cursor>> cs;
    const std::string seek = ikey(std::string(), kMaxSeq, true);  // before every key
    for (const FileMeta& m : in0) cs.emplace_back(new TableCursor(table(m.number, m.size), seek));
    for (const FileMeta& m : in1) cs.emplace_back(new TableCursor(table(m.number, m.size), seek));
    Merger mg(std::move(cs));
    std::string last_user;
    bool have_last = false;
    std::vector<FileMeta> outs = build_tables(out, [&](std::string* k, std::string* v) {
        while (mg.valid()) {
            Cursor* c = mg.top();
            const std::string& ik = c->key();
            const std::string u = user_of(ik);
            if (have_last && u == last_user) {  // an older version of a key already emitted
                mg.next();
                continue;
            }
            last_user = u;
            have_last = true;
            if (!is_value(ik) && !tombstone_needed(u, out)) {
                mg.next();
                continue;
            }
            *k = ik;
            *v = c->value();
            mg.next();
            return true;
        }
        return false;
    }, true);
    std::string e;
    put_varint(&e, 2);
    put_varint(&e, log_number_);
    put_varint(&e, 3);
    put_varint(&e, next_file_);
    put_varint(&e, 4);
    put_varint(&e, last_seq_);
    auto drop = [&](int l, const std::vector<FileMeta>& fs) {
        for (const FileMeta& m : fs) {
            put_varint(&e, 6);
            put_varint(&e, uint64_t(l));
            put_varint(&e, m.number);
            levels_[l].erase(std::remove_if(levels_[l].begin(), levels_[l].end(),
                                            [&](const FileMeta& x) { return x.number == m.number; }),
                             levels_[l].end());
        }
    };
    drop(level, in0);
    drop(out, in1);
    for (const FileMeta& m : outs) {
        put_varint(&e, 7);
        put_varint(&e, uint64_t(out));
        put_varint(&e, m.number);
        put_varint(&e, m.size);
        put_lenpref(&e, m.smallest);
        put_lenpref(&e, m.largest);
        levels_[out].push_back(m);
    }
    std::sort(levels_[out].begin(), levels_[out].end(),
              [](const FileMeta& a, const FileMeta& b) { return icmp(a.smallest, b.smallest) < 0; });
    append_edit(e);
    for (const auto* fs : {&in0, &in1})
        for (const FileMeta& m : *fs) {
            tables_.erase(m.number);
            table_used_.erase(m.number);
            ::unlink(fname(dir_, m.number, "ldb").c_str());
            ::unlink(fname(dir_, m.number, "sst").c_str());
        }
}

uint64_t DB::max_level_bytes(int level) const {
    uint64_t r = opt_.level1_bytes;
    for (int l = 1; l < level; ++l) r *= 10;
    return r;
}

void DB::maybe_compact() {
    for (;;) {
        if (int(levels_[0].size()) >= opt_.l0_compaction_trigger) {
            compact_level(0, true);
            continue;
        }
        int pick = -1;
        for (int l = 1; l < kLevels - 1; ++l)
            if (level_bytes(l) > max_level_bytes(l)) {
                pick = l;
                break;
            }
        if (pick < 0) return;
        compact_level(pick, false);
    }
}

void DB::write_locked(const WriteBatch& batch, bool sync) {
    if (closed_) fail("store is closed");
    if (batch.count() == 0) return;
    const uint64_t seq = last_seq_ + 1;
    std::string rep;
    put_fixed64(&rep, seq);
    put_fixed32(&rep, uint32_t(batch.count()));
    for (const auto& op : batch.ops()) {
        rep.push_back(char(op.put ? 1 : 0));
        put_lenpref(&rep, op.key);
        if (op.put) put_lenpref(&rep, op.value);
    }
    log_append(log_fd_, &log_block_off_, rep);
    if (sync && ::fdatasync(log_fd_) != 0) fail("fdatasync log");
    uint64_t s = seq;
    for (const auto& op : batch.ops()) {
        MemEntry& e = mem_[op.key];
        e.seq = s++;
        e.del = !op.put;
        e.value = op.value;
        mem_bytes_ += op.key.size() + op.value.size() + 32;
    }
    last_seq_ = seq + batch.count() - 1;
    if (mem_bytes_ >= opt_.write_buffer_size) {
        flush_memtable_locked();
        maybe_compact();
    }
}

void DB::write(const WriteBatch& batch, bool sync) {
    std::lock_guard<std::mutex> g(mu_);
    write_locked(batch, sync);
}
void DB::put(const std::string& k, const std::string& v, bool sync) {
    WriteBatch b;
    b.put(k, v);
    write(b, sync);
}
void DB::del(const std::string& k, bool sync) {
    WriteBatch b;
    b.del(k);
    write(b, sync);
}

bool DB::get(const std::string& key, std::string* value) {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) fail("store is closed");
    auto it = mem_.find(key);
    if (it != mem_.end()) {
        if (it->second.del) return false;
        *value = it->second.value;
        return true;
    }
    std::vector<const FileMeta*> l0;
    for (const FileMeta& m : levels_[0]) l0.push_back(&m);
    std::sort(l0.begin(), l0.end(), [](const FileMeta* a, const FileMeta* b) { return a->number > b->number; });
    for (const FileMeta* m : l0) {
        if (key < user_of(m->smallest) || user_of(m->largest) < key) continue;
        const int r = table(m->number, m->size)->get(key, value);
        if (r) return r == 1;
    }
    for (int l = 1; l < kLevels; ++l) {
        const auto& fs = levels_[l];
        size_t lo = 0, hi = fs.size();
        while (lo < hi) {  // first file whose largest user key >= key
            const size_t mid = (lo + hi) / 2;
            if (user_of(fs[mid].largest) < key) lo = mid + 1;
            else hi = mid;
        }
        if (lo == fs.size() || key < user_of(fs[lo].smallest)) continue;
        const int r = table(fs[lo].number, fs[lo].size)->get(key, value);
        if (r) return r == 1;
    }
    return false;
}

void DB::scan(const std::string& start, const std::string& end,
              const std::function<bool(const std::string&, const std::string&)>& f) {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) fail("store is closed");
    std::vector<std::unique_ptr<Cursor>> cs;
    std::vector<MemRow> rows;
    for (auto it = mem_.lower_bound(start); it != mem_.end(); ++it) {
        if (!end.empty() && it->first >= end) break;
        rows.push_back({ikey(it->first, it->second.seq, !it->second.del), it->second.value});
    }
    cs.emplace_back(new VecCursor(std::move(rows)));
    const std::string seek = ikey(start, kMaxSeq, true);
    for (int l = 0; l < kLevels; ++l)
        for (const FileMeta& m : levels_[l]) {
            if (user_of(m.largest) < start || (!end.empty() && user_of(m.smallest) >= end)) continue;
            cs.emplace_back(new TableCursor(table(m.number, m.size), seek));
        }
    Merger mg(std::move(cs));
    std::string last;
    bool have_last = false;
    while (mg.valid()) {
        Cursor* c = mg.top();
        const std::string u = user_of(c->key());
        if (!end.empty() && u >= end) break;
        if (!(have_last && u == last)) {
            last = u;
            have_last = true;
            if (is_value(c->key()) && !f(u, c->value())) break;
        }
        mg.next();
    }
}

void DB::flush_memtable() {
    std::lock_guard<std::mutex> g(mu_);
    flush_memtable_locked();
    maybe_compact();
}

void DB::compact_all() {
    std::lock_guard<std::mutex> g(mu_);
    flush_memtable_locked();
    int deepest = 1;
    for (int l = 1; l < kLevels; ++l)
        if (!levels_[l].empty()) deepest = l;
    for (int l = 0; l < deepest; ++l)
        if (!levels_[l].empty()) compact_level(l, true);
}

std::vector<int> DB::files_per_level() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int> r;
    for (int l = 0; l < kLevels; ++l) r.push_back(int(levels_[l].size()));
    return r;
}
uint64_t DB::last_sequence() {
    std::lock_guard<std::mutex> g(mu_);
    return last_seq_;
}
uint64_t DB::disk_bytes() {
    std::lock_guard<std::mutex> g(mu_);
    uint64_t s = 0;
    for (int l = 0; l < kLevels; ++l) s += level_bytes(l);
    return s;
}

}  // namespace ldb
}  // namespace nodexa
