// On-disk key-value store in the LevelDB format (SURVEY S5 block tree DB / S6 LevelDB).
//
// The reference keeps its block index (blocks/index/) and UTXO set (chainstate/) in LevelDB
// through CDBWrapper (src/dbwrapper.cpp:103-110: bloom filter policy, 10 bits per key, no
// compression; values XOR-ed with an 8-byte obfuscation key). This engine reads and writes the
// same directories file-for-file, so a reference datadir opens here without -reindex and a
// datadir written here opens in the reference:
//
//   CURRENT          name of the live manifest
//   MANIFEST-NNNNNN  log of version edits: comparator, log / next-file numbers, last sequence,
//                    table files added / removed per level
//   NNNNNN.log       write-ahead log of write batches (32 KiB blocks, CRC32C-framed records)
//   NNNNNN.ldb/.sst  sorted tables: prefix-compressed 4 KiB data blocks with restart points, a
//                    bloom filter block over user keys, metaindex, index block, 48-byte footer
//
// What is engine-specific (behaviour, not format): the memtable holds only the newest version
// of each key (no snapshots are needed by the node); opening always folds the write-ahead log
// into a level-0 table and starts a fresh manifest (as the reference's leveldb does without
// reuse_logs); compaction is leveled (level-0 file-count trigger, 10 MiB x 10^(L-1) level
// budgets) and runs inline on the writing thread. Snappy-compressed blocks are read (older
// datadirs, or ones written with compression on) but never written.
#pragma once

#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace nodexa {
namespace ldb {

struct Options {
    bool create_if_missing = true;
    bool error_if_exists = false;
    size_t write_buffer_size = 4u << 20;  // memtable bytes before it becomes a level-0 table
    size_t block_size = 4096;             // data block target (uncompressed)
    int block_restart_interval = 16;
    size_t max_file_size = 2u << 20;      // table files written by compaction
    int bloom_bits_per_key = 10;          // 0: tables carry no filter block
    int l0_compaction_trigger = 4;
    uint64_t level1_bytes = 10ull << 20;  // level L holds up to level1_bytes x 10^(L-1)
    size_t max_open_files = 512;          // open table files kept (least recently used closed first)
};

class WriteBatch {
public:
    void put(const std::string& key, const std::string& value) { ops_.push_back({true, key, value}); }
    void del(const std::string& key) { ops_.push_back({false, key, std::string()}); }
    size_t count() const { return ops_.size(); }
    void clear() { ops_.clear(); }
    struct Op {
        bool put;
        std::string key, value;
    };
    const std::vector<Op>& ops() const { return ops_; }

private:
    std::vector<Op> ops_;
};

struct FileMeta {
    uint64_t number = 0, size = 0;
    std::string smallest, largest;  // internal keys
};

class Table;

class DB {
public:
    // Opens (or creates) the store in `dir`; throws std::runtime_error on corruption or I/O errors.
    static std::unique_ptr<DB> open(const std::string& dir, const Options& opt = Options());
    ~DB();
    DB(const DB&) = delete;
    DB& operator=(const DB&) = delete;

    bool get(const std::string& key, std::string* value);
    void put(const std::string& key, const std::string& value, bool sync = false);
    void del(const std::string& key, bool sync = false);
    void write(const WriteBatch& batch, bool sync = false);
    // Visits the live entries with start <= key < end (an empty `end` is unbounded) in key
    // order; stops early when `f` returns false.
    void scan(const std::string& start, const std::string& end,
              const std::function<bool(const std::string&, const std::string&)>& f);
    // Memtable to a table, then every level merged into one sorted run at the deepest level used.
    void compact_all();
    void flush_memtable();
    std::vector<int> files_per_level();
    uint64_t last_sequence();
    uint64_t disk_bytes();
    void close();

private:
    explicit DB(const std::string& dir, const Options& opt);
    struct MemEntry {
        uint64_t seq;
        bool del;
        std::string value;
    };
    void recover();
    void replay_log(uint64_t number);
    void write_locked(const WriteBatch& batch, bool sync);
    void new_log();
    void flush_memtable_locked();
    void maybe_compact();
    void compact_level(int level, bool whole_level);
    void write_snapshot_manifest();
    void append_edit(const std::string& edit);
    void delete_obsolete();
    std::shared_ptr<Table> table(uint64_t number, uint64_t size);
    std::vector<FileMeta> build_tables(int level_hint, const std::function<bool(std::string*, std::string*)>& next,
                                       bool split);
    bool tombstone_needed(const std::string& user_key, int out_level) const;
    uint64_t level_bytes(int level) const;
    uint64_t max_level_bytes(int level) const;

    std::string dir_;
    Options opt_;
    std::mutex mu_;
    int lock_fd_ = -1;
    std::string open_key_;  // canonical path in the process's set of open stores
    int log_fd_ = -1;
    int manifest_fd_ = -1;
    uint64_t log_number_ = 0, manifest_number_ = 0, next_file_ = 2, last_seq_ = 0;
    uint32_t log_block_off_ = 0, manifest_block_off_ = 0;
    std::map<std::string, MemEntry> mem_;
    size_t mem_bytes_ = 0;
    std::vector<FileMeta> levels_[7];
    std::map<uint64_t, std::shared_ptr<Table>> tables_;  // open tables (cursors may hold others alive)
    std::map<uint64_t, uint64_t> table_used_;             // last use stamp of each open table
    uint64_t table_clock_ = 0;
    size_t compact_cursor_[7] = {0, 0, 0, 0, 0, 0, 0};
    bool closed_ = false;
};

// Removes a store directory's files (DestroyDB).
void destroy(const std::string& dir);

// Format pieces exposed for tests and for the chain-format codecs.
uint32_t crc32c(const void* data, size_t n, uint32_t init = 0);
uint32_t crc_mask(uint32_t crc);
uint32_t bloom_hash(const std::string& key);
bool snappy_uncompress(const char* in, size_t n, std::string* out);

}  // namespace ldb
}  // namespace nodexa
