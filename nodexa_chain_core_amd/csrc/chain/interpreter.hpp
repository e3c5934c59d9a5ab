// Script evaluation and transaction signature checking.
//
// Parity: EvalScript / VerifyScript / VerifyWitnessProgram (src/script/interpreter.cpp:289,1546),
// SignatureHash legacy + BIP143 (interpreter.cpp:1150-1380), TransactionSignatureChecker (CheckSig /
// CheckLockTime / CheckSequence), CScriptNum (src/script/script.h:221-340), the BIP66 DER and
// low-S rules, FindAndDelete, and Clore's OP_CLORE_ASSET (0xc0): GetOp returns everything after it
// as one data element (src/script/script.h:580-586) and EvalScript treats it as a no-op
// (interpreter.cpp:1119-1121). Flags and error names are the reference's
// (src/script/interpreter.h:39-114, script_error.h), so src/test/data/script_tests.json,
// sighash.json and tx_valid.json / tx_invalid.json run unchanged (tests/test_script.py).
//
// Signatures go through a SigChecker. The default checks each one on the host (secp256k1.cpp);
// block validation collects them in a batch for the GPU (hip/kernels/secp256k1_verify.hip) by
// running the scripts with a deferring checker (see ScriptCheckBatch).
#pragma once

#include <functional>
#include <string>
#include <vector>

#include "primitives.hpp"

namespace nodexa {

enum ScriptFlags : u32 {
    SCRIPT_VERIFY_NONE = 0,
    SCRIPT_VERIFY_P2SH = 1u << 0,
    SCRIPT_VERIFY_STRICTENC = 1u << 1,
    SCRIPT_VERIFY_DERSIG = 1u << 2,
    SCRIPT_VERIFY_LOW_S = 1u << 3,
    SCRIPT_VERIFY_NULLDUMMY = 1u << 4,
    SCRIPT_VERIFY_SIGPUSHONLY = 1u << 5,
    SCRIPT_VERIFY_MINIMALDATA = 1u << 6,
    SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_NOPS = 1u << 7,
    SCRIPT_VERIFY_CLEANSTACK = 1u << 8,
    SCRIPT_VERIFY_CHECKLOCKTIMEVERIFY = 1u << 9,
    SCRIPT_VERIFY_CHECKSEQUENCEVERIFY = 1u << 10,
    SCRIPT_VERIFY_WITNESS = 1u << 11,
    SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM = 1u << 12,
    SCRIPT_VERIFY_MINIMALIF = 1u << 13,
    SCRIPT_VERIFY_NULLFAIL = 1u << 14,
    SCRIPT_VERIFY_WITNESS_PUBKEYTYPE = 1u << 15,
};
// MANDATORY_SCRIPT_VERIFY_FLAGS / STANDARD_SCRIPT_VERIFY_FLAGS (src/policy/policy.h)
constexpr u32 kMandatoryScriptFlags = SCRIPT_VERIFY_P2SH;
constexpr u32 kStandardScriptFlags =
    SCRIPT_VERIFY_P2SH | SCRIPT_VERIFY_DERSIG | SCRIPT_VERIFY_STRICTENC | SCRIPT_VERIFY_MINIMALDATA |
    SCRIPT_VERIFY_NULLDUMMY | SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_NOPS | SCRIPT_VERIFY_CLEANSTACK |
    SCRIPT_VERIFY_MINIMALIF | SCRIPT_VERIFY_NULLFAIL | SCRIPT_VERIFY_CHECKLOCKTIMEVERIFY |
    SCRIPT_VERIFY_CHECKSEQUENCEVERIFY | SCRIPT_VERIFY_LOW_S | SCRIPT_VERIFY_WITNESS |
    SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM | SCRIPT_VERIFY_WITNESS_PUBKEYTYPE;

enum class ScriptError {
    OK, UNKNOWN_ERROR, EVAL_FALSE, OP_RETURN, SCRIPT_SIZE, PUSH_SIZE, OP_COUNT, STACK_SIZE, SIG_COUNT,
    PUBKEY_COUNT, VERIFY, EQUALVERIFY, CHECKMULTISIGVERIFY, CHECKSIGVERIFY, NUMEQUALVERIFY, BAD_OPCODE,
    DISABLED_OPCODE, INVALID_STACK_OPERATION, INVALID_ALTSTACK_OPERATION, UNBALANCED_CONDITIONAL,
    NEGATIVE_LOCKTIME, UNSATISFIED_LOCKTIME, SIG_HASHTYPE, SIG_DER, MINIMALDATA, SIG_PUSHONLY, SIG_HIGH_S,
    SIG_NULLDUMMY, PUBKEYTYPE, CLEANSTACK, MINIMALIF, NULLFAIL, DISCOURAGE_UPGRADABLE_NOPS,
    DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM, WITNESS_PROGRAM_WRONG_LENGTH, WITNESS_PROGRAM_WITNESS_EMPTY,
    WITNESS_PROGRAM_MISMATCH, WITNESS_MALLEATED, WITNESS_MALLEATED_P2SH, WITNESS_UNEXPECTED,
    WITNESS_PUBKEYTYPE,
};
const char* script_error_name(ScriptError e);

enum class SigVersion { BASE = 0, WITNESS_V0 = 1 };

enum SigHashType : int { SIGHASH_ALL = 1, SIGHASH_NONE = 2, SIGHASH_SINGLE = 3, SIGHASH_ANYONECANPAY = 0x80 };

// Script limits (src/script/script.h:28-44)
constexpr size_t kMaxScriptElementSize = 520;
constexpr int kMaxOpsPerScript = 201;
constexpr int kMaxPubkeysPerMultisig = 20;
constexpr size_t kMaxScriptSize = 10000;
constexpr size_t kMaxStackSize = 1000;
constexpr u32 kLocktimeThreshold = 500000000;
constexpr u8 OP_CLORE_ASSET = 0xc0;

// One opcode (and its push data) at `pc`; false on a truncated push (GetScriptOp).
bool script_get_op(const Bytes& s, size_t& pc, u8& opcode, Bytes* data);
bool script_is_push_only(const Bytes& s);
bool script_is_p2sh(const Bytes& s);
bool script_is_witness_program(const Bytes& s, int& version, Bytes& program);
// Legacy sigop count (GetSigOpCount(false)) and the accurate P2SH form over the redeem script.
unsigned script_sigop_count(const Bytes& s, bool accurate);

// BIP143 midstate hashes of one transaction (PrecomputedTransactionData).
struct PrecomputedTx {
    Uint256 prevouts, sequence, outputs;
    bool ready = false;
    explicit PrecomputedTx(const Transaction& tx);
    PrecomputedTx() = default;
};

Uint256 signature_hash(const Bytes& script_code, const Transaction& tx, unsigned n_in, int hash_type, Amount amount,
                       SigVersion sigversion, const PrecomputedTx* cache = nullptr);

// Signature / locktime oracle used by EvalScript.
class SigChecker {
public:
    virtual ~SigChecker() = default;
    virtual bool check_sig(const Bytes& sig, const Bytes& pubkey, const Bytes& script_code, SigVersion sv) const {
        (void)sig; (void)pubkey; (void)script_code; (void)sv;
        return false;
    }
    virtual bool check_lock_time(int64_t n) const { (void)n; return false; }
    virtual bool check_sequence(int64_t n) const { (void)n; return false; }
};

// A signature check deferred for a batch: message hash, DER signature (hash type stripped) and
// public key, as the GPU batch verifier takes them.
struct PendingSig {
    Uint256 msg;
    Bytes sig;
    Bytes pubkey;
};

class TxSigChecker : public SigChecker {
public:
    TxSigChecker(const Transaction* tx, unsigned n_in, Amount amount, const PrecomputedTx* cache = nullptr)
        : tx_(tx), n_in_(n_in), amount_(amount), cache_(cache) {}
    bool check_sig(const Bytes& sig, const Bytes& pubkey, const Bytes& script_code, SigVersion sv) const override;
    bool check_lock_time(int64_t n) const override;
    bool check_sequence(int64_t n) const override;
    // Batch mode: check_sig records the signature in `pending` and answers true (the caller
    // re-runs the input on the host if the batch rejects any of its signatures). Only
    // valid for scripts whose outcome cannot depend on a signature failing, i.e. for blocks,
    // where any failing signature invalidates the block anyway.
    std::vector<PendingSig>* pending = nullptr;
    // Signature cache (sigcache.hpp): STORE remembers every signature that verifies (mempool
    // acceptance); USE answers from the cache first and erases what it hits (block validation,
    // CachingTransactionSignatureChecker with store = false).
    enum class CacheMode : u8 { NONE, STORE, USE };
    CacheMode sigcache = CacheMode::NONE;

protected:
    const Transaction* tx_;
    unsigned n_in_;
    Amount amount_;
    const PrecomputedTx* cache_;
};

bool eval_script(std::vector<Bytes>& stack, const Bytes& script, u32 flags, const SigChecker& checker,
                 SigVersion sv, ScriptError* err);
bool verify_script(const Bytes& script_sig, const Bytes& script_pubkey, const std::vector<Bytes>* witness, u32 flags,
                   const SigChecker& checker, ScriptError* err);

// Context-free transaction checks (CheckTransaction, src/consensus/tx_verify.cpp:169; the asset
// null-data rules are not included). Returns "" or the reference's reject reason.
// CheckTransaction. With `asset_params`, also the asset rules of CheckTransaction (assets.hpp),
// under the given deployment flags (block_check: called from CheckBlock; mempool_check: from ATMP).
namespace assets {
struct Params;
struct Flags;
}  // namespace assets
std::string check_transaction(const Transaction& tx, bool check_duplicate_inputs = true,
                              const assets::Params* asset_params = nullptr, const assets::Flags* flags = nullptr,
                              bool block_check = false, bool mempool_check = false);
constexpr Amount kMaxMoney = Amount(1300000000) * COIN;  // src/amount.h:29

// DER / pubkey encoding rules exposed for tests and policy.
bool is_valid_signature_encoding(const Bytes& sig);
bool is_low_der_signature(const Bytes& sig);
bool is_compressed_or_uncompressed_pubkey(const Bytes& pk);

}  // namespace nodexa
