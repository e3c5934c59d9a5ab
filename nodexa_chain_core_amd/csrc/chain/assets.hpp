// Asset layer: asset names, asset scripts, the asset state (metadata, balances,
// qualifier tags, address / global restrictions, verifier strings) and the consensus checks that
// ConnectBlock and AcceptToMemoryPool apply to asset transactions.
//
// Parity (behaviour, written for this engine):
//  - names: IsAssetNameValid / IsTypeCheckNameValid / GetParentName (src/assets/assets.cpp:44-420)
//  - scripts: CScript::IsAssetScript, IsNullAsset* (src/script/script.cpp:233-360), the CNewAsset /
//    CAssetTransfer / CReissueAsset / CNullAssetTxData encodings (src/assets/assettypes.h:59-330) and
//    their ConstructTransaction forms (P2PKH + OP_CLORE_ASSET + push("rvn" type payload) + OP_DROP)
//  - context-free checks: the asset part of CheckTransaction (src/consensus/tx_verify.cpp:169-560)
//    with VerifyNewAsset / VerifyNewUniqueAsset / VerifyReissueAsset / ... (src/assets/assets.cpp)
//  - contextual checks: Consensus::CheckTxAssets (tx_verify.cpp:607-915), ContextualCheck*Asset,
//    the verifier-string checks (assets.cpp:4863-5206)
//  - state updates: AddCoins / SpendCoin with an assets cache (src/coins.cpp:99-380), CAssetsCache
//    (src/assets/assets.cpp:1667-2273). Every change is journalled; the journal is the block's
//    asset undo record, so DisconnectBlock restores the exact prior state.
//  - verifier strings: LibBoolEE (src/LibBoolEE.cpp), as a recursive-descent evaluator with the
//    same operators (| & ! parentheses, 1/0 constants) and the same error cases.
#pragma once

#include <functional>
#include <map>
#include <optional>
#include <set>
#include <string>
#include <vector>

#include "primitives.hpp"

namespace nodexa {

struct Coin;

namespace assets {

constexpr int64_t kCoin = 100000000;
constexpr int kMaxUnit = 8;
constexpr int64_t kOwnerAmount = kCoin;
constexpr int64_t kUniqueAmount = kCoin;
constexpr int64_t kQualifierMin = kCoin;
constexpr int64_t kQualifierMax = 10 * kCoin;
constexpr u8 kOpAsset = 0xc0;

enum class Type { ROOT, SUB, UNIQUE, MSGCHANNEL, OWNER, VOTE, REISSUE, QUALIFIER, SUB_QUALIFIER, RESTRICTED,
                  NULL_ADD_QUALIFIER, INVALID };
const char* type_name(Type t);

// IsAssetNameValid: the type of a valid name, INVALID (with a reason in *err) otherwise.
Type name_type(const std::string& name, std::string* err = nullptr);
inline bool name_valid(const std::string& name) { return name_type(name) != Type::INVALID; }
std::string parent_name(const std::string& name);  // GetParentName ("" if invalid)
bool is_owner_name(const std::string& name);        // "NAME!"
bool amount_fits_units(int64_t amount, int units);  // CheckAmountWithUnits

// ---- LibBoolEE-compatible verifier expressions
// Evaluates `expr` (whitespace ignored) with the variable values in `vals`; throws
// std::runtime_error on a syntax error or an unknown variable.
bool bool_expr(const std::string& expr, const std::map<std::string, bool>& vals);
std::string strip_verifier(const std::string& verifier);  // no whitespace, no '#'
std::set<std::string> verifier_qualifiers(const std::string& stripped);
// CheckVerifierString: syntax, length (<= 80 stripped) and qualifier-name checks.
bool check_verifier(const std::string& verifier, std::set<std::string>& found, std::string& err);

// ---- scripts
enum class OutKind { NONE, NEW, OWNER, TRANSFER, REISSUE };
struct AssetOut {
    OutKind kind = OutKind::NONE;
    u8 h160[20] = {0};    // the P2PKH destination in front of OP_CLORE_ASSET
    std::string name;
    int64_t amount = 0;
    int units = 0;        // new: 0..8; reissue: -1 = unchanged
    int reissuable = 0;
    int has_ipfs = 0;
    std::string ipfs;     // 34-byte multihash (0x12 0x20 ...) or 32-byte txid, raw
    std::string message;  // transfer message, same raw forms
    int64_t expire = 0;
};
// IsAssetScript: the kind and where the payload starts (0 if not an asset script).
OutKind asset_script_kind(const Bytes& spk, size_t* payload_at = nullptr);
// Decodes an asset script (false if it is none, or does not deserialize).
bool parse_asset_out(const Bytes& spk, AssetOut& out);
// GetAssetAmountFromScript (owner tokens count OWNER_ASSET_AMOUNT).
bool asset_amount(const Bytes& spk, int64_t& amount);
// CScript::IsUnspendable, with the asset rules (OP_CLORE_ASSET first, or an asset amount of 0).
bool script_unspendable(const Bytes& spk);

enum class NullKind { NONE, TAG, GLOBAL, VERIFIER };
NullKind null_kind(const Bytes& spk);
bool parse_null_tag(const Bytes& spk, std::string& name, int& flag, u8 h160[20]);
bool parse_null_global(const Bytes& spk, std::string& name, int& flag);
bool parse_null_verifier(const Bytes& spk, std::string& verifier);

Bytes script_new(const u8 h160[20], const AssetOut& a);  // 'q'
Bytes script_owner(const u8 h160[20], const std::string& name);  // 'o', name includes '!'
Bytes script_transfer(const u8 h160[20], const std::string& name, int64_t amount, const std::string& message = "",
                      int64_t expire = 0);
Bytes script_reissue(const u8 h160[20], const std::string& name, int64_t amount, int units, int reissuable,
                     const std::string& ipfs);
Bytes script_null_tag(const u8 h160[20], const std::string& name, int flag);
Bytes script_null_global(const std::string& name, int flag);
Bytes script_null_verifier(const std::string& verifier);

// ---- consensus parameters (burn amounts and burn scripts per network, src/chainparams.cpp)
struct Params {
    int64_t burn_root = 500 * kCoin, burn_reissue = 100 * kCoin, burn_sub = 100 * kCoin, burn_unique = 5 * kCoin,
            burn_msgchannel = 100 * kCoin, burn_qualifier = 1000 * kCoin, burn_subqualifier = 100 * kCoin,
            burn_restricted = 1500 * kCoin, burn_tag = kCoin / 10;
    Bytes spk_root, spk_reissue, spk_sub, spk_unique, spk_msgchannel, spk_qualifier, spk_subqualifier,
        spk_restricted, spk_tag, spk_global;
    bool testnet = false;
    int64_t burn_amount(Type t) const;
    const Bytes* burn_script(Type t) const;
};

// Deployment state for the block (or mempool) being checked.
struct Flags {
    bool assets = false;            // DEPLOYMENT_ASSETS
    bool msg_restricted = false;    // DEPLOYMENT_MSG_REST_ASSETS (messaging + restricted assets)
    bool enforce_values = false;    // DEPLOYMENT_ENFORCE_VALUE
    bool coinbase_assets = false;   // DEPLOYMENT_COINBASE_ASSETS
};

// ---- transaction classification (CTransaction::IsNewAsset / IsReissueAsset / ...)
enum class TxKind { NONE, NEW, NEW_UNIQUE, NEW_MSGCHANNEL, NEW_QUALIFIER, NEW_RESTRICTED, REISSUE };
TxKind tx_kind(const Transaction& tx);

// Context-free asset rules of CheckTransaction: "" or the reject reason.
std::string check_tx_structure(const Transaction& tx, const Params& p, const Flags& f, bool block_check,
                               bool mempool_check);

struct Meta {
    std::string name;
    int64_t amount = 0;
    int units = 0;
    int reissuable = 0;
    int has_ipfs = 0;
    std::string ipfs;
    int height = 0;
    Uint256 block;
};

using AddrKey = std::pair<std::string, std::string>;  // (asset name, 20-byte hash as a string)

// The asset state with a change journal (the undo record of a block).
class State {
public:
    const Meta* find(const std::string& name) const;
    bool exists(const std::string& name) const { return find(name) != nullptr; }
    int64_t balance(const std::string& name, const u8 h160[20]) const;
    bool has_tag(const std::string& qualifier, const u8 h160[20]) const;
    bool frozen(const std::string& restricted, const u8 h160[20]) const;
    bool global_frozen(const std::string& restricted) const { return global_.count(restricted) != 0; }
    const std::string* verifier(const std::string& restricted) const;

    const std::map<std::string, Meta>& metas() const { return meta_; }
    const std::map<AddrKey, int64_t>& balances() const { return bal_; }
    const std::set<AddrKey>& tags() const { return tags_; }
    const std::set<AddrKey>& restrictions() const { return frozen_; }
    const std::set<std::string>& global_restrictions() const { return global_; }
    const std::map<std::string, std::string>& verifiers() const { return verifier_; }

    // journalled mutations
    void set_meta(const Meta& m);
    void erase_meta(const std::string& name);
    void add_balance(const std::string& name, const u8 h160[20], int64_t delta);
    void set_tag(const std::string& q, const u8 h160[20], bool on);
    void set_frozen(const std::string& r, const u8 h160[20], bool on);
    void set_global(const std::string& r, bool on);
    void set_verifier(const std::string& r, const std::string& v);

    // journal control: mark() -> apply changes -> journal_since(mark) is their undo record
    size_t mark() const { return journal_.size(); }
    Bytes journal_since(size_t m) const;
    void rollback_to(size_t m);                 // undo the changes after mark m
    void clear_journal() { journal_.clear(); }
    bool undo(const Bytes& record);             // revert a record produced by journal_since

    Bytes serialize() const;                    // snapshot (assets.dat)
    bool deserialize(const Bytes& b);
    Uint256 best_block;

    // Incremental persistence (store/chaindb.hpp assets records): every entry changed since
    // clear_dirty() as (kind, a, b, current value or nullptr when absent); load_entry() inserts a
    // stored value without marking it changed.
    void for_each_dirty(const std::function<void(u8, const std::string&, const std::string&, const Bytes*)>& f) const;
    void clear_dirty() { dirty_.clear(); }
    void mark_all_dirty();                      // every entry changed (an imported state's first flush)
    size_t dirty_count() const { return dirty_.size(); }
    bool load_entry(u8 kind, const std::string& a, const std::string& b, const Bytes& value);
    void reset() { *this = State(); }

private:
    struct Op {
        u8 kind;  // 0 meta, 1 balance, 2 tag, 3 frozen, 4 global, 5 verifier
        std::string a, b;
        bool had = false;
        Bytes old;  // serialized previous value
    };
    void log(u8 kind, const std::string& a, const std::string& b);
    void restore(const Op& op);
    std::map<std::string, Meta> meta_;
    std::map<AddrKey, int64_t> bal_;
    std::set<AddrKey> tags_;
    std::set<AddrKey> frozen_;
    std::set<std::string> global_;
    std::map<std::string, std::string> verifier_;
    std::vector<Op> journal_;
    std::set<std::pair<u8, AddrKey>> dirty_;
};

// Consensus::CheckTxAssets against `st` (spent: the coin of every input). "" or reject reason.
// `pending_names` (mempool): asset names already being created by pool transactions.
std::string check_tx_contextual(const Transaction& tx, const std::vector<const Coin*>& spent, const State& st,
                                const Flags& f, const std::set<std::string>* pending_names = nullptr);
// AddCoins / SpendCoin asset effects of a connected transaction.
void apply_tx(const Transaction& tx, const std::vector<Coin>& spent, int height, const Uint256& block_hash,
              State& st);

// Hex / base58 display form of an IPFS hash or txid (EncodeAssetData).
std::string encode_asset_data(const std::string& raw);
// DecodeAssetData: "Qm..." (46 chars) -> 34 raw bytes, 64 hex chars -> 32 raw bytes, else "".
std::string decode_asset_data(const std::string& s);

}  // namespace assets
}  // namespace nodexa
