// UTXO set, block undo data and block connection (SURVEY S3 ConnectBlock / S4 UTXO set / S9).
//
// Parity: Coin / CCoinsViewCache (src/coins.h:34-323), ConnectBlock / DisconnectBlock
// (src/validation.cpp:10052, 9479) for the native chain rules — inputs present and unspent,
// coinbase maturity (COINBASE_MATURITY 100, src/consensus/consensus.h:27), value ranges and fees,
// BIP68 sequence locks (CalculateSequenceLocks), sigop cost (MAX_BLOCK_SIGOPS_COST 80000,
// GetTransactionSigOpCost) and every input script under the block's flags (GetBlockScriptFlags,
// validation.cpp:10005: P2SH, DERSIG, CLTV, CSV, WITNESS and NULLDUMMY are enabled on every
// network). Undo records use the reference's rev?????.dat encoding (CBlockUndo of CTxUndo, each
// coin as VARINT(height*2+coinbase) [VARINT(0)] + CTxOutCompressor, src/undo.h, compressor.h),
// written with the blk-file framing plus the sha256d(block hash || undo) checksum.
//
// Assets: with `ConnectOptions::assets` set, every transaction also passes
// Consensus::CheckTxAssets against the asset state and its asset effects are applied (assets.hpp);
// the state changes are journalled and returned as the block's asset undo record.
//
// Signatures: with `defer_sigs` set, connect_block runs every script with a deferring checker and
// returns the signatures for the GPU batch verifier (ops/secp.py); the caller then re-runs only
// the inputs whose signatures the batch rejected on the host (see ChainState in chain/state.py).
#pragma once

#include <functional>
#include <string>
#include <unordered_map>
#include <vector>

#include "assets.hpp"
#include "interpreter.hpp"
#include "primitives.hpp"

namespace nodexa {

constexpr int kCoinbaseMaturity = 100;
constexpr int64_t kMaxBlockSigopsCost = 80000;
constexpr u32 kBlockScriptFlags = SCRIPT_VERIFY_P2SH | SCRIPT_VERIFY_DERSIG | SCRIPT_VERIFY_CHECKLOCKTIMEVERIFY |
                                  SCRIPT_VERIFY_CHECKSEQUENCEVERIFY | SCRIPT_VERIFY_WITNESS | SCRIPT_VERIFY_NULLDUMMY;

struct Coin {
    TxOut out;
    u32 height = 0;
    bool coinbase = false;
};

struct OutPointHasher {
    size_t operator()(const OutPoint& o) const noexcept {
        u64 h;
        std::memcpy(&h, o.hash.data, 8);
        return size_t(h ^ (u64(o.n) * 0x9E3779B97F4A7C15ULL));
    }
};
struct OutPointEq {
    bool operator()(const OutPoint& a, const OutPoint& b) const noexcept {
        return a.n == b.n && std::memcmp(a.hash.data, b.hash.data, 32) == 0;
    }
};

class CoinsView {
public:
    const Coin* find(const OutPoint& o) const;
    void add(const OutPoint& o, Coin c);
    bool spend(const OutPoint& o, Coin* moved = nullptr);
    size_t size() const { return map_.size(); }
    Uint256 best_block;
    // Snapshot persistence (chainstate/coins.dat): written to path.new, fsynced and renamed.
    void save(const std::string& path) const;
    bool load(const std::string& path);  // false if absent or corrupt (the view is then empty)
    // Incremental persistence, the analogue of CCoinsViewDB::BatchWrite (src/txdb.cpp:91-): a
    // flush appends one checksummed record holding only the outputs added or spent since the
    // previous flush (plus the new best block) to a journal (chainstate/coins.log) and fsyncs it,
    // so flush cost follows the change set, not the UTXO set. Records carry a sequence number and
    // the snapshot the one of the last record folded into it; start-up loads the snapshot and
    // replays the newer complete records (a torn tail record from a crash is cut off). compact()
    // folds the journal into a fresh snapshot.
    void append_journal(const std::string& journal);
    bool load_with_journal(const std::string& snapshot, const std::string& journal);
    void compact(const std::string& snapshot, const std::string& journal);
    size_t dirty() const { return dirty_.size(); }
    u64 journal_seq = 0;      // records written (or replayed) so far
    size_t replayed = 0;      // records applied by the last load_with_journal
    // gettxoutsetinfo: (number of unspent outputs, transactions with unspent outputs, total value,
    // hash_serialized_2 over the best block and the coins in (txid, n) order, bogosize).
    struct Stats {
        u64 txouts = 0, transactions = 0, bogosize = 0;
        Amount total = 0;
        Uint256 hash;
    };
    Stats stats() const;
    template <class F>
    void for_each(F&& f) const {
        for (auto& kv : map_) f(kv.first, kv.second);
    }
    // The change set since the last flush: f(outpoint, coin or nullptr when spent).
    template <class F>
    void for_each_dirty(F&& f) const {
        for (auto& kv : dirty_) f(kv.first, kv.second ? find(kv.first) : nullptr);
    }
    void clear_dirty() { dirty_.clear(); }
    void reset() {
        map_.clear();
        dirty_.clear();
        best_block = Uint256();
    }
    void insert_clean(const OutPoint& o, Coin c) { map_[o] = std::move(c); }  // loaded state, not a change
    void reserve(size_t n) { map_.reserve(n); }

private:
    std::unordered_map<OutPoint, Coin, OutPointHasher, OutPointEq> map_;
    std::unordered_map<OutPoint, bool, OutPointHasher, OutPointEq> dirty_;  // since the last flush
};

struct TxUndo {
    std::vector<Coin> prev;  // spent coins in input order
};
struct BlockUndo {
    std::vector<TxUndo> vtxundo;  // one per non-coinbase transaction
};
Bytes serialize_block_undo(const BlockUndo& u);
BlockUndo deserialize_block_undo(const Bytes& b);

// CompressAmount / DecompressAmount and the script compressor (src/compressor.cpp)
u64 compress_amount(u64 n);
u64 decompress_amount(u64 x);
// The chainstate database's coin record (Coin::Serialize, src/coins.h:58-72: VARINT(height*2 +
// coinbase) then CTxOutCompressor) and the serialize.h VARINT (MSB base-128, +1 per continuation).
Bytes serialize_coin_db(const Coin& c);
bool deserialize_coin_db(const u8* p, size_t n, Coin& c);
void append_varint(Bytes& out, u64 n);
bool parse_varint(const u8*& p, const u8* end, u64& n);

struct ConnectOptions {
    u32 script_flags = kBlockScriptFlags;
    bool check_scripts = true;
    bool defer_sigs = false;   // collect signatures for a batch verifier instead of checking them
    bool sigcache = true;      // skip (and drop) signatures the mempool already verified (sigcache.hpp)
    bool sequence_locks = true;
    // median time past of the block at `height` of this block's chain (BIP68 time locks)
    std::function<int64_t(int)> mtp_at;
    int64_t block_mtp = 0;     // MTP of the previous block (the block's lock-time reference)
    // Script-check threads (CCheckQueue / -par): the UTXO pass stays serial, the collected
    // input checks then run on this many threads (1 = inline). The first failing input in
    // block order decides the reject reason, as with a serial run.
    int threads = 1;
    // Asset layer (null: asset outputs are plain outputs and no asset rule is applied)
    assets::State* assets = nullptr;
    assets::Flags asset_flags;
    Uint256 block_hash;
};

struct ConnectResult {
    bool ok = true;
    std::string reject;
    int dos = 0;
    Amount fees = 0;
    int64_t sigop_cost = 0;
    std::vector<PendingSig> sigs;            // with defer_sigs: every signature to verify
    std::vector<std::pair<u32, u32>> sig_at;  // (tx index, input index) of each entry of sigs
    Bytes asset_undo;                          // the asset journal of the block (with opt.assets)
};

// Applies `block` (at `height`) to `view`; on failure the view is left unchanged.
ConnectResult connect_block(const Block& block, int height, CoinsView& view, const ConnectOptions& opt,
                            BlockUndo& undo);
// Re-runs one input's scripts with host signature checks (the fallback for a rejected batch).
bool verify_input_host(const Transaction& tx, unsigned n_in, const Coin& coin, u32 flags, ScriptError* err);
// Reverts `block` with its undo data; false if the data do not match the view. With `assets`, the
// block's asset undo record is reverted too.
bool disconnect_block(const Block& block, const BlockUndo& undo, CoinsView& view, assets::State* assets = nullptr,
                      const Bytes* asset_undo = nullptr);

// GetLegacySigOpCount: inaccurate sigops of every scriptSig and scriptPubKey.
int64_t tx_legacy_sigops(const Transaction& tx);
// Transaction sigop cost (GetTransactionSigOpCost) given its spent coins (one per input; may be
// empty only for a coinbase).
int64_t tx_sigop_cost(const Transaction& tx, const std::vector<const Coin*>& spent, u32 flags);

}  // namespace nodexa
