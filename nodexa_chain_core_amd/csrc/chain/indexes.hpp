// Optional chain indexes: -txindex, -addressindex, -spentindex, -timestampindex.
//
// Parity (behaviour): the index writes of ConnectBlock / DisconnectBlock
// (src/validation.cpp:9518-9910 and 10234-10482) and their readers GetTransaction (txindex),
// GetAddressIndex / GetAddressUnspent / GetSpentIndex / GetTimestampIndex
// (src/validation.cpp:1122-1205), queried by the addressindex RPCs (src/rpc/misc.cpp:880-1460),
// getblockdeltas / getblockhashes (src/rpc/blockchain.cpp). The reference keeps these in
// LevelDB; here they are resident hash maps (a node with 288 GB of host-visible memory per GPU
// box keeps them in RAM) snapshotted to chainstate/indexes.dat together with the UTXO set.
//
// Address keys: type 1 = P2PKH (and P2PK, by hash160 of the key, and asset outputs, by their
// P2PKH destination), type 2 = P2SH. Asset outputs are indexed under their asset name with the
// asset amount, CLORE outputs under "CLORE" (the reference's default asset name).
#pragma once

#include <functional>
#include <map>
#include <optional>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "coins.hpp"

namespace nodexa {

struct AddrDelta {
    int height = 0;
    u32 tx_index = 0;  // position of the transaction in its block
    Uint256 txid;
    u32 index = 0;     // output index, or input index when spending
    bool spending = false;
    int64_t amount = 0;
};

struct AddrUnspent {
    Uint256 txid;
    u32 index = 0;
    int64_t amount = 0;
    Bytes script;
    int height = 0;
};

struct SpentInfo {
    Uint256 txid;      // spending transaction
    u32 input = 0;
    int height = 0;
    int64_t amount = 0;
    int addr_type = 0;
    u8 h160[20] = {0};
};

// (address type, hash160) of a scriptPubKey for the address index, plus the asset it carries
// ("CLORE" for plain outputs). False if the script has no indexable address.
bool index_address(const Bytes& spk, int& type, u8 h160[20], std::string& asset, int64_t& amount, int64_t value);

class ChainIndexes {
public:
    bool txindex = false, addressindex = false, spentindex = false, timestampindex = false;
    Uint256 best_block;

    // `file` / `data_pos`: where the block's data lives (blk file, offset after the framing); the
    // txindex records of the change journal address transactions by them (CDiskTxPos), -1 = none.
    void connect(const Block& block, int height, const Uint256& hash, const BlockUndo& undo, int file = -1,
                 u32 data_pos = 0);
    void disconnect(const Block& block, int height, const Uint256& hash, const BlockUndo& undo);

    // Change journal in the reference's blocks/index record layout (CBlockTreeDB, txdb.cpp:250-440):
    // 't' txid -> CDiskTxPos, 'a' CAddressIndexKey -> amount, 'u' CAddressUnspentKey ->
    // CAddressUnspentValue, 'p' CSpentIndexKey -> CSpentIndexValue, 's' CTimestampIndexKey -> 0,
    // 'z' block hash -> timestamp. With `journal` on, connect / disconnect append every record they
    // add (value) or remove (nullopt); take_changes() hands them over for one write batch.
    bool journal = false;
    using Change = std::pair<std::string, std::optional<std::string>>;
    std::vector<Change> take_changes() { return std::move(changes_); }
    size_t pending_changes() const { return changes_.size(); }
    // Rebuilds the resident maps from such records (`tx_block_at` maps a (file, data_pos) to the
    // block hash stored there). False on a malformed record.
    bool load_records(const std::function<void(const std::function<void(const std::string&, const std::string&)>&)>& scan,
                      const std::function<bool(int, u32, Uint256*)>& tx_block_at);

    const Uint256* tx_block(const Uint256& txid) const;
    // asset "*" = every asset; start/end = inclusive height range (0, 0 = all)
    std::vector<std::pair<std::string, AddrDelta>> deltas(int type, const u8 h160[20], const std::string& asset,
                                                          int start = 0, int end = 0) const;
    std::vector<std::pair<std::string, AddrUnspent>> unspent(int type, const u8 h160[20], const std::string& asset) const;
    const SpentInfo* spent(const Uint256& txid, u32 n) const;
    std::vector<Uint256> timestamps(u32 low, u32 high) const;  // low <= time < high, in time order

    size_t size_txindex() const { return tx_.size(); }

    Bytes serialize() const;
    bool deserialize(const Bytes& b);

private:
    using Key = std::string;  // type byte + hash160 + asset name
    static Key key(int type, const u8 h160[20], const std::string& asset);
    struct OutKeyHash {
        size_t operator()(const std::pair<Uint256, u32>& k) const noexcept {
            u64 h;
            std::memcpy(&h, k.first.data, 8);
            return size_t(h ^ (u64(k.second) * 0x9E3779B97F4A7C15ULL));
        }
    };
    struct U256Hash {
        size_t operator()(const Uint256& u) const noexcept {
            u64 h;
            std::memcpy(&h, u.data, 8);
            return size_t(h);
        }
    };
    struct U256Eq {
        bool operator()(const Uint256& a, const Uint256& b) const noexcept { return std::memcmp(a.data, b.data, 32) == 0; }
    };
    struct OutEq {
        bool operator()(const std::pair<Uint256, u32>& a, const std::pair<Uint256, u32>& b) const noexcept {
            return a.second == b.second && std::memcmp(a.first.data, b.first.data, 32) == 0;
        }
    };
    void rec_put(std::string k, std::string v) {
        if (journal) changes_.emplace_back(std::move(k), std::move(v));
    }
    void rec_erase(std::string k) {
        if (journal) changes_.emplace_back(std::move(k), std::nullopt);
    }
    std::vector<Change> changes_;
    std::unordered_map<Uint256, Uint256, U256Hash, U256Eq> tx_;
    std::map<Key, std::vector<AddrDelta>> deltas_;
    std::map<Key, std::map<std::pair<Uint256, u32>, AddrUnspent>> unspent_;
    std::unordered_map<std::pair<Uint256, u32>, SpentInfo, OutKeyHash, OutEq> spent_;
    std::multimap<u32, Uint256> time_;
};

}  // namespace nodexa
