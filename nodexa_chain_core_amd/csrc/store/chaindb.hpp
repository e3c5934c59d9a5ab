// The reference's chain databases on the LevelDB-format store: the UTXO set
// (CCoinsViewDB, chainstate/) and the block tree (CBlockTreeDB, blocks/index/), key for key
// (src/txdb.cpp:23-38) and with CDBWrapper's value obfuscation (src/dbwrapper.cpp:150-172).
//
//   chainstate   'C' + txid + VARINT(n) -> Coin (VARINT(height*2+coinbase), CTxOutCompressor)
//                'B' -> best block hash;  'H' -> head blocks of an interrupted flush
//   blocks/index 'b' + hash -> CDiskBlockIndex (chain.h:403-433);  'f' + i32 -> CBlockFileInfo;
//                'l' -> last block file;  'R' -> reindexing;  'F' + name -> flag
//   both         "\x0e\x00obfuscate_key" -> the 8-byte XOR key (serialized as a vector)
//
// A flush of the UTXO change set is one atomic, synced write batch (coins and 'B' together), so
// no 'H' marker is needed; a reference datadir that carries one (a crash mid-flush there) is
// reported to the caller, which rebuilds instead of trusting a half-written set.
#pragma once

#include <string>
#include <vector>

#include "../chain/coins.hpp"
#include "../chain/indexes.hpp"
#include "ldb.hpp"

namespace nodexa {
namespace chaindb {

// Reads the store's obfuscation key; a new (empty) store gets a fresh random one written, as
// CDBWrapper does; a non-empty store without one keeps the all-zero key (pre-obfuscation data).
std::string obfuscation_key(ldb::DB& db, bool create);
void xor_obf(std::string& v, const std::string& key);

struct CoinsLoad {
    bool have_best = false;
    bool head_blocks = false;  // 'H' present: the last flush did not complete
    size_t coins = 0, bad = 0;
};
// CCoinsViewDB load: every 'C' record into the view (replacing its contents) and 'B'.
CoinsLoad coins_load(CoinsView& view, ldb::DB& db, const std::string& obf);
// CCoinsViewDB::BatchWrite: the view's change set (puts and erases) plus 'B' in one synced
// batch; clears the change set. Returns the number of coin records written or erased. With
// `assets`, the asset state's changed entries and its best block go into the same batch
// (this engine's keys: 0x01 kind name key -> value, "\x02assets.best"), so the UTXO set and the
// asset state on disk always describe the same block.
size_t coins_flush(CoinsView& view, ldb::DB& db, const std::string& obf, bool sync,
                   assets::State* assets = nullptr);
// the asset state from those records; false if they are malformed or absent
bool assets_load(assets::State& st, ldb::DB& db, const std::string& obf);
std::string coin_key(const OutPoint& o);

// A reference datadir's asset state: CAssetsDB (assets/: 'A' name -> CDatabasedAssetData, 'B'
// (name, address) -> CAmount; src/assets/assetdb.cpp:17-41) and CRestrictedDB (assets/restricted:
// 'V' verifier strings, 'T' (address, qualifier) tags, 'R' (address, name) frozen addresses, 'G'
// global freezes; src/assets/restricteddb.cpp:10-100) read into `st` (replacing its contents;
// addresses become their 20-byte hashes, as this engine keys them). The reverse indexes ('C',
// 'Q'), the mempool reissue state ('Z') and the undo records ('U') are not needed for the state.
struct RefAssetsLoad {
    size_t metas = 0, balances = 0, tags = 0, restrictions = 0, globals = 0, verifiers = 0, bad = 0;
};
RefAssetsLoad assets_import_reference(assets::State& st, ldb::DB& assets_db, ldb::DB* restricted_db);

// CDiskBlockIndex
struct DiskIndex {
    Uint256 hash;
    int height = 0;
    u32 status = 0;
    u32 ntx = 0;
    int file = -1;
    u32 data_pos = 0, undo_pos = 0;
    Bytes header;  // this engine's header serialization (KawPow headers carry nHeight)
};
enum : u32 {
    BLOCK_VALID_TREE = 2,
    BLOCK_VALID_TRANSACTIONS = 3,
    BLOCK_VALID_CHAIN = 4,
    BLOCK_VALID_SCRIPTS = 5,
    BLOCK_VALID_MASK = 7,
    BLOCK_HAVE_DATA = 8,
    BLOCK_HAVE_UNDO = 16,
    BLOCK_FAILED_VALID = 32,
    BLOCK_FAILED_CHILD = 64,
};
// value of a 'b' record; `kawpow_time` is the activation time that selects the header form
std::string encode_disk_index(const DiskIndex& d, u32 kawpow_time, int client_version = 4000000);
bool decode_disk_index(const std::string& v, u32 kawpow_time, DiskIndex* d);
// every 'b' record, de-obfuscated and decoded (hash from the key), in key order
std::vector<DiskIndex> load_block_index(ldb::DB& db, const std::string& obf, u32 kawpow_time, size_t* bad);

// Optional indexes (-txindex/-addressindex/-spentindex/-timestampindex) in blocks/index: the
// journal of `ix` plus the block it describes ("\x00nodexa.indexes.best", this engine's key) in
// one batch; the load rebuilds the resident maps ('t' positions resolved through `block_at`).
size_t indexes_flush(ChainIndexes& ix, ldb::DB& db, const std::string& obf, bool sync);
bool indexes_load(ChainIndexes& ix, ldb::DB& db, const std::string& obf,
                  const std::function<bool(int, u32, Uint256*)>& block_at, bool* have_best);
// drops every index record (a rebuild with other flags)
void indexes_purge(ldb::DB& db);

struct FileInfo {
    u32 blocks = 0, size = 0, undo_size = 0, height_first = 0, height_last = 0;
    u64 time_first = 0, time_last = 0;
};
std::string encode_file_info(const FileInfo& f);
bool decode_file_info(const std::string& v, FileInfo* f);

}  // namespace chaindb
}  // namespace nodexa
