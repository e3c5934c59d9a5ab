// Script interpreter: see interpreter.hpp.
#include "interpreter.hpp"
#include "sigcache.hpp"

#include "assets.hpp"

#include <algorithm>
#include <climits>
#include <set>

#include "../crypto/hashes.hpp"
#include "../crypto/secp256k1.hpp"
#include "../crypto/sha256.hpp"
#include "script.hpp"

namespace nodexa {

namespace {

// opcodes used by the interpreter (src/script/script.h:47-200)
enum : u8 {
    kOP_0 = 0x00, kOP_PUSHDATA1 = 0x4c, kOP_PUSHDATA2 = 0x4d, kOP_PUSHDATA4 = 0x4e, kOP_1NEGATE = 0x4f,
    kOP_RESERVED = 0x50, kOP_1 = 0x51, kOP_16 = 0x60, kOP_NOP = 0x61, kOP_VER = 0x62, kOP_IF = 0x63,
    kOP_NOTIF = 0x64, kOP_VERIF = 0x65, kOP_VERNOTIF = 0x66, kOP_ELSE = 0x67, kOP_ENDIF = 0x68,
    kOP_VERIFY = 0x69, kOP_RETURN = 0x6a, kOP_TOALTSTACK = 0x6b, kOP_FROMALTSTACK = 0x6c, kOP_2DROP = 0x6d,
    kOP_2DUP = 0x6e, kOP_3DUP = 0x6f, kOP_2OVER = 0x70, kOP_2ROT = 0x71, kOP_2SWAP = 0x72, kOP_IFDUP = 0x73,
    kOP_DEPTH = 0x74, kOP_DROP = 0x75, kOP_DUP = 0x76, kOP_NIP = 0x77, kOP_OVER = 0x78, kOP_PICK = 0x79,
    kOP_ROLL = 0x7a, kOP_ROT = 0x7b, kOP_SWAP = 0x7c, kOP_TUCK = 0x7d, kOP_CAT = 0x7e, kOP_SUBSTR = 0x7f,
    kOP_LEFT = 0x80, kOP_RIGHT = 0x81, kOP_SIZE = 0x82, kOP_INVERT = 0x83, kOP_AND = 0x84, kOP_OR = 0x85,
    kOP_XOR = 0x86, kOP_EQUAL = 0x87, kOP_EQUALVERIFY = 0x88, kOP_1ADD = 0x8b, kOP_1SUB = 0x8c,
    kOP_2MUL = 0x8d, kOP_2DIV = 0x8e, kOP_NEGATE = 0x8f, kOP_ABS = 0x90, kOP_NOT = 0x91,
    kOP_0NOTEQUAL = 0x92, kOP_ADD = 0x93, kOP_SUB = 0x94, kOP_MUL = 0x95, kOP_DIV = 0x96, kOP_MOD = 0x97,
    kOP_LSHIFT = 0x98, kOP_RSHIFT = 0x99, kOP_BOOLAND = 0x9a, kOP_BOOLOR = 0x9b, kOP_NUMEQUAL = 0x9c,
    kOP_NUMEQUALVERIFY = 0x9d, kOP_NUMNOTEQUAL = 0x9e, kOP_LESSTHAN = 0x9f, kOP_GREATERTHAN = 0xa0,
    kOP_LESSTHANOREQUAL = 0xa1, kOP_GREATERTHANOREQUAL = 0xa2, kOP_MIN = 0xa3, kOP_MAX = 0xa4,
    kOP_WITHIN = 0xa5, kOP_RIPEMD160 = 0xa6, kOP_SHA1 = 0xa7, kOP_SHA256 = 0xa8, kOP_HASH160 = 0xa9,
    kOP_HASH256 = 0xaa, kOP_CODESEPARATOR = 0xab, kOP_CHECKSIG = 0xac, kOP_CHECKSIGVERIFY = 0xad,
    kOP_CHECKMULTISIG = 0xae, kOP_CHECKMULTISIGVERIFY = 0xaf, kOP_NOP1 = 0xb0, kOP_CHECKLOCKTIMEVERIFY = 0xb1,
    kOP_CHECKSEQUENCEVERIFY = 0xb2, kOP_NOP4 = 0xb3, kOP_NOP10 = 0xb9,
};

constexpr u32 kSequenceFinal = 0xffffffffu;
constexpr u32 kSeqLocktimeDisable = 1u << 31;
constexpr u32 kSeqLocktimeType = 1u << 22;
constexpr u32 kSeqLocktimeMask = 0x0000ffffu;

struct ScriptNumError {};

// CScriptNum: little-endian sign-magnitude integers of at most `max_size` bytes.
int64_t scriptnum_decode(const Bytes& v, bool require_minimal, size_t max_size = 4) {
    if (v.size() > max_size) throw ScriptNumError{};
    if (require_minimal && !v.empty()) {
        if ((v.back() & 0x7f) == 0 && (v.size() <= 1 || (v[v.size() - 2] & 0x80) == 0)) throw ScriptNumError{};
    }
    if (v.empty()) return 0;
    int64_t r = 0;
    for (size_t i = 0; i < v.size(); ++i) r |= int64_t(v[i]) << (8 * i);
    if (v.back() & 0x80) return -int64_t(r & ~(int64_t(0x80) << (8 * (v.size() - 1))));
    return r;
}

Bytes scriptnum_encode(int64_t value) {
    Bytes r;
    if (value == 0) return r;
    const bool neg = value < 0;
    uint64_t a = neg ? uint64_t(-(value + 1)) + 1 : uint64_t(value);
    while (a) {
        r.push_back(u8(a & 0xff));
        a >>= 8;
    }
    if (r.back() & 0x80) r.push_back(neg ? 0x80 : 0);
    else if (neg) r.back() |= 0x80;
    return r;
}

int scriptnum_getint(int64_t v) {
    if (v > INT_MAX) return INT_MAX;
    if (v < INT_MIN) return INT_MIN;
    return int(v);
}

bool cast_to_bool(const Bytes& v) {
    for (size_t i = 0; i < v.size(); ++i) {
        if (v[i] != 0) return !(i == v.size() - 1 && v[i] == 0x80);  // negative zero is false
    }
    return false;
}

bool check_minimal_push(const Bytes& data, u8 opcode) {
    if (data.empty()) return opcode == kOP_0;
    if (data.size() == 1 && data[0] >= 1 && data[0] <= 16) return opcode == kOP_1 + (data[0] - 1);
    if (data.size() == 1 && data[0] == 0x81) return opcode == kOP_1NEGATE;
    if (data.size() <= 75) return opcode == data.size();
    if (data.size() <= 255) return opcode == kOP_PUSHDATA1;
    if (data.size() <= 65535) return opcode == kOP_PUSHDATA2;
    return true;
}

bool is_defined_hashtype(const Bytes& sig) {
    if (sig.empty()) return false;
    const int t = sig.back() & ~SIGHASH_ANYONECANPAY;
    return t >= SIGHASH_ALL && t <= SIGHASH_SINGLE;
}

bool set_err(ScriptError* e, ScriptError v) {
    if (e) *e = v;
    return v == ScriptError::OK;
}

bool check_signature_encoding(const Bytes& sig, u32 flags, ScriptError* err) {
    if (sig.empty()) return true;  // empty signature: a compact way to provide an invalid one
    if ((flags & (SCRIPT_VERIFY_DERSIG | SCRIPT_VERIFY_LOW_S | SCRIPT_VERIFY_STRICTENC)) &&
        !is_valid_signature_encoding(sig))
        return set_err(err, ScriptError::SIG_DER);
    if ((flags & SCRIPT_VERIFY_LOW_S) && !is_low_der_signature(sig)) return set_err(err, ScriptError::SIG_HIGH_S);
    if ((flags & SCRIPT_VERIFY_STRICTENC) && !is_defined_hashtype(sig)) return set_err(err, ScriptError::SIG_HASHTYPE);
    return true;
}

bool check_pubkey_encoding(const Bytes& pk, u32 flags, SigVersion sv, ScriptError* err) {
    if ((flags & SCRIPT_VERIFY_STRICTENC) && !is_compressed_or_uncompressed_pubkey(pk))
        return set_err(err, ScriptError::PUBKEYTYPE);
    if ((flags & SCRIPT_VERIFY_WITNESS_PUBKEYTYPE) && sv == SigVersion::WITNESS_V0 &&
        !(pk.size() == 33 && (pk[0] == 2 || pk[0] == 3)))
        return set_err(err, ScriptError::WITNESS_PUBKEYTYPE);
    return true;
}

// CScript() << data: the minimal push opcode for `data`
Bytes push_script(const Bytes& d) {
    Bytes s;
    if (d.size() < kOP_PUSHDATA1) {
        s.push_back(u8(d.size()));
    } else if (d.size() <= 0xff) {
        s.push_back(kOP_PUSHDATA1);
        s.push_back(u8(d.size()));
    } else if (d.size() <= 0xffff) {
        s.push_back(kOP_PUSHDATA2);
        s.push_back(u8(d.size()));
        s.push_back(u8(d.size() >> 8));
    } else {
        s.push_back(kOP_PUSHDATA4);
        for (int i = 0; i < 4; ++i) s.push_back(u8(d.size() >> (8 * i)));
    }
    s.insert(s.end(), d.begin(), d.end());
    return s;
}

// FindAndDelete (interpreter.cpp): remove every op-aligned occurrence of `b` from `s`.
int find_and_delete(Bytes& s, const Bytes& b) {
    int found = 0;
    if (b.empty()) return found;
    Bytes result;
    size_t pc = 0, pc2 = 0;
    u8 op;
    do {
        result.insert(result.end(), s.begin() + pc2, s.begin() + pc);
        while (s.size() - pc >= b.size() && std::equal(b.begin(), b.end(), s.begin() + pc)) {
            pc += b.size();
            ++found;
        }
        pc2 = pc;
    } while (script_get_op(s, pc, op, nullptr));
    if (found > 0) {
        result.insert(result.end(), s.begin() + pc2, s.end());
        s.swap(result);
    }
    return found;
}

bool is_disabled(u8 op) {
    switch (op) {
        case kOP_CAT: case kOP_SUBSTR: case kOP_LEFT: case kOP_RIGHT: case kOP_INVERT: case kOP_AND: case kOP_OR:
        case kOP_XOR: case kOP_2MUL: case kOP_2DIV: case kOP_MUL: case kOP_DIV: case kOP_MOD: case kOP_LSHIFT:
        case kOP_RSHIFT:
            return true;
        default:
            return false;
    }
}

Uint256 hash_bytes(const Bytes& b) {
    Uint256 h;
    sha256d(b.data(), b.size(), h.data);
    return h;
}

}  // namespace

const char* script_error_name(ScriptError e) {
    static const char* names[] = {
        "OK", "UNKNOWN_ERROR", "EVAL_FALSE", "OP_RETURN", "SCRIPT_SIZE", "PUSH_SIZE", "OP_COUNT", "STACK_SIZE",
        "SIG_COUNT", "PUBKEY_COUNT", "VERIFY", "EQUALVERIFY", "CHECKMULTISIGVERIFY", "CHECKSIGVERIFY",
        "NUMEQUALVERIFY", "BAD_OPCODE", "DISABLED_OPCODE", "INVALID_STACK_OPERATION", "INVALID_ALTSTACK_OPERATION",
        "UNBALANCED_CONDITIONAL", "NEGATIVE_LOCKTIME", "UNSATISFIED_LOCKTIME", "SIG_HASHTYPE", "SIG_DER",
        "MINIMALDATA", "SIG_PUSHONLY", "SIG_HIGH_S", "SIG_NULLDUMMY", "PUBKEYTYPE", "CLEANSTACK", "MINIMALIF",
        "NULLFAIL", "DISCOURAGE_UPGRADABLE_NOPS", "DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM",
        "WITNESS_PROGRAM_WRONG_LENGTH", "WITNESS_PROGRAM_WITNESS_EMPTY", "WITNESS_PROGRAM_MISMATCH",
        "WITNESS_MALLEATED", "WITNESS_MALLEATED_P2SH", "WITNESS_UNEXPECTED", "WITNESS_PUBKEYTYPE"};
    return names[int(e)];
}

bool script_get_op(const Bytes& s, size_t& pc, u8& opcode, Bytes* data) {
    opcode = 0xff;
    if (data) data->clear();
    if (pc >= s.size()) return false;
    const u8 op = s[pc++];
    if (op <= kOP_PUSHDATA4) {
        size_t n = 0;
        if (op < kOP_PUSHDATA1) {
            n = op;
        } else if (op == kOP_PUSHDATA1) {
            if (s.size() - pc < 1) return false;
            n = s[pc++];
        } else if (op == kOP_PUSHDATA2) {
            if (s.size() - pc < 2) return false;
            n = size_t(s[pc]) | size_t(s[pc + 1]) << 8;
            pc += 2;
        } else {
            if (s.size() - pc < 4) return false;
            n = load_le32(s.data() + pc);
            pc += 4;
        }
        if (s.size() - pc < n) return false;
        if (data) data->assign(s.begin() + pc, s.begin() + pc + n);
        pc += n;
    }
    if (op == OP_CLORE_ASSET) {  // everything after the asset marker is data, not opcodes
        if (data) data->assign(s.begin() + pc, s.end());
        pc = s.size();
    }
    opcode = op;
    return true;
}

bool script_is_push_only(const Bytes& s) {
    size_t pc = 0;
    while (pc < s.size()) {
        u8 op;
        if (!script_get_op(s, pc, op, nullptr)) return false;
        if (op > kOP_16) return false;
    }
    return true;
}

bool script_is_p2sh(const Bytes& s) {
    return s.size() == 23 && s[0] == kOP_HASH160 && s[1] == 0x14 && s[22] == kOP_EQUAL;
}

bool script_is_witness_program(const Bytes& s, int& version, Bytes& program) {
    if (s.size() < 4 || s.size() > 42) return false;
    if (s[0] != kOP_0 && (s[0] < kOP_1 || s[0] > kOP_16)) return false;
    if (size_t(s[1]) + 2 != s.size()) return false;
    version = s[0] == kOP_0 ? 0 : s[0] - (kOP_1 - 1);
    program.assign(s.begin() + 2, s.end());
    return true;
}

unsigned script_sigop_count(const Bytes& s, bool accurate) {
    unsigned n = 0;
    size_t pc = 0;
    u8 last = 0xff, op;
    while (pc < s.size()) {
        if (!script_get_op(s, pc, op, nullptr)) break;
        if (op == kOP_CHECKSIG || op == kOP_CHECKSIGVERIFY) {
            ++n;
        } else if (op == kOP_CHECKMULTISIG || op == kOP_CHECKMULTISIGVERIFY) {
            if (accurate && last >= kOP_1 && last <= kOP_16) n += last - (kOP_1 - 1);
            else n += kMaxPubkeysPerMultisig;
        }
        last = op;
    }
    return n;
}

bool is_valid_signature_encoding(const Bytes& sig) {
    // BIP66: 0x30 [total] 0x02 [R-len] [R] 0x02 [S-len] [S] [sighash]
    if (sig.size() < 9 || sig.size() > 73) return false;
    if (sig[0] != 0x30) return false;
    if (sig[1] != sig.size() - 3) return false;
    const size_t len_r = sig[3];
    if (5 + len_r >= sig.size()) return false;
    const size_t len_s = sig[5 + len_r];
    if (len_r + len_s + 7 != sig.size()) return false;
    if (sig[2] != 0x02) return false;
    if (len_r == 0) return false;
    if (sig[4] & 0x80) return false;
    if (len_r > 1 && sig[4] == 0x00 && !(sig[5] & 0x80)) return false;
    if (sig[len_r + 4] != 0x02) return false;
    if (len_s == 0) return false;
    if (sig[len_r + 6] & 0x80) return false;
    if (len_s > 1 && sig[len_r + 6] == 0x00 && !(sig[len_r + 7] & 0x80)) return false;
    return true;
}

bool is_low_der_signature(const Bytes& sig) {
    if (!is_valid_signature_encoding(sig)) return false;
    secp::Scalar r, s;
    if (!secp::sig_parse_der_lax(sig.data(), sig.size() - 1, r, s)) return false;
    return !secp::sc_is_high(s);
}

bool is_compressed_or_uncompressed_pubkey(const Bytes& pk) {
    if (pk.size() < 33) return false;
    if (pk[0] == 0x04) return pk.size() == 65;
    if (pk[0] == 0x02 || pk[0] == 0x03) return pk.size() == 33;
    return false;
}

// ------------------------------------------------------------------ signature hashes
PrecomputedTx::PrecomputedTx(const Transaction& tx) {
    Writer a, b, c;
    for (auto& in : tx.vin) {
        a.u256(in.prevout.hash);
        a.u32_(in.prevout.n);
        b.u32_(in.sequence);
    }
    for (auto& o : tx.vout) {
        c.i64_(o.value);
        c.var_bytes(o.script_pubkey);
    }
    prevouts = hash_bytes(a.buf);
    sequence = hash_bytes(b.buf);
    outputs = hash_bytes(c.buf);
    ready = true;
}

Uint256 signature_hash(const Bytes& script_code, const Transaction& tx, unsigned n_in, int hash_type, Amount amount,
                       SigVersion sigversion, const PrecomputedTx* cache) {
    const int base = hash_type & 0x1f;
    const bool anyone = hash_type & SIGHASH_ANYONECANPAY;
    if (sigversion == SigVersion::WITNESS_V0) {
        Uint256 hp, hs, ho;  // zero unless committed
        PrecomputedTx local;
        if (!cache || !cache->ready) {
            local = PrecomputedTx(tx);
            cache = &local;
        }
        if (!anyone) hp = cache->prevouts;
        if (!anyone && base != SIGHASH_SINGLE && base != SIGHASH_NONE) hs = cache->sequence;
        if (base != SIGHASH_SINGLE && base != SIGHASH_NONE) {
            ho = cache->outputs;
        } else if (base == SIGHASH_SINGLE && n_in < tx.vout.size()) {
            Writer w;
            w.i64_(tx.vout[n_in].value);
            w.var_bytes(tx.vout[n_in].script_pubkey);
            ho = hash_bytes(w.buf);
        }
        Writer w;
        w.i32_(tx.version);
        w.u256(hp);
        w.u256(hs);
        w.u256(tx.vin[n_in].prevout.hash);
        w.u32_(tx.vin[n_in].prevout.n);
        w.var_bytes(script_code);
        w.i64_(amount);
        w.u32_(tx.vin[n_in].sequence);
        w.u256(ho);
        w.u32_(tx.lock_time);
        w.i32_(hash_type);
        return hash_bytes(w.buf);
    }
    Uint256 one;
    one.data[0] = 1;
    if (n_in >= tx.vin.size()) return one;
    if (base == SIGHASH_SINGLE && n_in >= tx.vout.size()) return one;
    // CTransactionSignatureSerializer::SerializeScriptCode: the script without OP_CODESEPARATORs.
    // As in the reference, the length prefix is size - separators and the bytes stop where the op
    // walk stops (a truncated push ends the walk early, so the prefix can overstate the bytes).
    auto write_code = [&](Writer& w) {
        size_t pc = 0, seps = 0;
        u8 op;
        while (script_get_op(script_code, pc, op, nullptr))
            if (op == kOP_CODESEPARATOR) ++seps;
        w.compact_size(script_code.size() - seps);
        size_t seg = 0;
        pc = 0;
        while (script_get_op(script_code, pc, op, nullptr)) {
            if (op == kOP_CODESEPARATOR) {
                w.raw(script_code.data() + seg, pc - 1 - seg);
                seg = pc;
            }
        }
        if (seg != script_code.size()) w.raw(script_code.data() + seg, pc - seg);
    };
    Writer w;
    w.i32_(tx.version);
    const size_t nin = anyone ? 1 : tx.vin.size();
    w.compact_size(nin);
    for (size_t k = 0; k < nin; ++k) {
        const size_t i = anyone ? n_in : k;
        w.u256(tx.vin[i].prevout.hash);
        w.u32_(tx.vin[i].prevout.n);
        if (i != n_in) w.compact_size(0);
        else write_code(w);
        if (i != n_in && (base == SIGHASH_SINGLE || base == SIGHASH_NONE)) w.u32_(0);
        else w.u32_(tx.vin[i].sequence);
    }
    const size_t nout = base == SIGHASH_NONE ? 0 : (base == SIGHASH_SINGLE ? n_in + 1 : tx.vout.size());
    w.compact_size(nout);
    for (size_t i = 0; i < nout; ++i) {
        if (base == SIGHASH_SINGLE && i != n_in) {
            w.i64_(-1);
            w.compact_size(0);
        } else {
            w.i64_(tx.vout[i].value);
            w.var_bytes(tx.vout[i].script_pubkey);
        }
    }
    w.u32_(tx.lock_time);
    w.i32_(hash_type);
    return hash_bytes(w.buf);
}

bool TxSigChecker::check_sig(const Bytes& sig_in, const Bytes& pubkey, const Bytes& script_code, SigVersion sv) const {
    // CPubKey(vch).IsValid(): a known header and the matching length
    if (pubkey.empty()) return false;
    const u8 h = pubkey[0];
    const size_t want = (h == 2 || h == 3) ? 33 : (h == 4 || h == 6 || h == 7) ? 65 : 0;
    if (!want || pubkey.size() != want) return false;
    if (sig_in.empty()) return false;
    const int hash_type = sig_in.back();
    const Bytes sig(sig_in.begin(), sig_in.end() - 1);
    const Uint256 msg = signature_hash(script_code, *tx_, n_in_, hash_type, amount_, sv, cache_);
    if (sigcache != CacheMode::NONE && SigCache::instance().get(msg.data, pubkey, sig, sigcache == CacheMode::USE))
        return true;  // verified when the transaction entered the mempool
    if (pending) {
        pending->push_back(PendingSig{msg, sig, pubkey});
        return true;
    }
    const bool ok = secp::verify_der(pubkey.data(), pubkey.size(), sig.data(), sig.size(), msg.data);
    if (ok && sigcache == CacheMode::STORE) SigCache::instance().put(msg.data, pubkey, sig);
    return ok;
}

bool TxSigChecker::check_lock_time(int64_t n) const {
    const int64_t tl = tx_->lock_time;
    if (!((tl < kLocktimeThreshold && n < kLocktimeThreshold) || (tl >= kLocktimeThreshold && n >= kLocktimeThreshold)))
        return false;
    if (n > tl) return false;
    if (tx_->vin[n_in_].sequence == kSequenceFinal) return false;
    return true;
}

bool TxSigChecker::check_sequence(int64_t n) const {
    const int64_t ts = tx_->vin[n_in_].sequence;
    if (u32(tx_->version) < 2) return false;
    if (ts & kSeqLocktimeDisable) return false;
    const u32 mask = kSeqLocktimeType | kSeqLocktimeMask;
    const int64_t tsm = ts & mask, nm = n & mask;
    if (!((tsm < kSeqLocktimeType && nm < kSeqLocktimeType) || (tsm >= kSeqLocktimeType && nm >= kSeqLocktimeType)))
        return false;
    return nm <= tsm;
}

// ------------------------------------------------------------------ EvalScript
bool eval_script(std::vector<Bytes>& stack, const Bytes& script, u32 flags, const SigChecker& checker,
                 SigVersion sv, ScriptError* err) {
    static const Bytes kFalse, kTrue(1, 1);
    set_err(err, ScriptError::UNKNOWN_ERROR);
    if (script.size() > kMaxScriptSize) return set_err(err, ScriptError::SCRIPT_SIZE);
    size_t pc = 0, begin_code = 0;
    std::vector<bool> exec;
    std::vector<Bytes> alt;
    int op_count = 0;
    const bool minimal = flags & SCRIPT_VERIFY_MINIMALDATA;
    auto top = [&](int i) -> Bytes& { return stack[stack.size() + i]; };
    auto pop = [&] { stack.pop_back(); };
    try {
        while (pc < script.size()) {
            const bool f_exec = std::find(exec.begin(), exec.end(), false) == exec.end();
            u8 op;
            Bytes push;
            if (!script_get_op(script, pc, op, &push)) return set_err(err, ScriptError::BAD_OPCODE);
            if (push.size() > kMaxScriptElementSize) return set_err(err, ScriptError::PUSH_SIZE);
            if (op > kOP_16 && ++op_count > kMaxOpsPerScript) return set_err(err, ScriptError::OP_COUNT);
            if (is_disabled(op)) return set_err(err, ScriptError::DISABLED_OPCODE);

            if (f_exec && op <= kOP_PUSHDATA4) {
                if (minimal && !check_minimal_push(push, op)) return set_err(err, ScriptError::MINIMALDATA);
                stack.push_back(std::move(push));
            } else if (f_exec || (kOP_IF <= op && op <= kOP_ENDIF)) {
                switch (op) {
                    case kOP_1NEGATE:
                    case kOP_1: case kOP_1 + 1: case kOP_1 + 2: case kOP_1 + 3: case kOP_1 + 4: case kOP_1 + 5:
                    case kOP_1 + 6: case kOP_1 + 7: case kOP_1 + 8: case kOP_1 + 9: case kOP_1 + 10:
                    case kOP_1 + 11: case kOP_1 + 12: case kOP_1 + 13: case kOP_1 + 14: case kOP_16:
                        stack.push_back(scriptnum_encode(int(op) - int(kOP_1 - 1)));
                        break;
                    case kOP_NOP:
                        break;
                    case kOP_CHECKLOCKTIMEVERIFY: {
                        if (!(flags & SCRIPT_VERIFY_CHECKLOCKTIMEVERIFY)) {
                            if (flags & SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_NOPS)
                                return set_err(err, ScriptError::DISCOURAGE_UPGRADABLE_NOPS);
                            break;
                        }
                        if (stack.size() < 1) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        const int64_t lt = scriptnum_decode(top(-1), minimal, 5);
                        if (lt < 0) return set_err(err, ScriptError::NEGATIVE_LOCKTIME);
                        if (!checker.check_lock_time(lt)) return set_err(err, ScriptError::UNSATISFIED_LOCKTIME);
                        break;
                    }
                    case kOP_CHECKSEQUENCEVERIFY: {
                        if (!(flags & SCRIPT_VERIFY_CHECKSEQUENCEVERIFY)) {
                            if (flags & SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_NOPS)
                                return set_err(err, ScriptError::DISCOURAGE_UPGRADABLE_NOPS);
                            break;
                        }
                        if (stack.size() < 1) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        const int64_t seq = scriptnum_decode(top(-1), minimal, 5);
                        if (seq < 0) return set_err(err, ScriptError::NEGATIVE_LOCKTIME);
                        if (seq & kSeqLocktimeDisable) break;
                        if (!checker.check_sequence(seq)) return set_err(err, ScriptError::UNSATISFIED_LOCKTIME);
                        break;
                    }
                    case kOP_NOP1: case kOP_NOP4: case kOP_NOP4 + 1: case kOP_NOP4 + 2: case kOP_NOP4 + 3:
                    case kOP_NOP4 + 4: case kOP_NOP4 + 5: case kOP_NOP10:
                        if (flags & SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_NOPS)
                            return set_err(err, ScriptError::DISCOURAGE_UPGRADABLE_NOPS);
                        break;
                    case kOP_IF:
                    case kOP_NOTIF: {
                        bool value = false;
                        if (f_exec) {
                            if (stack.size() < 1) return set_err(err, ScriptError::UNBALANCED_CONDITIONAL);
                            const Bytes& v = top(-1);
                            if (sv == SigVersion::WITNESS_V0 && (flags & SCRIPT_VERIFY_MINIMALIF)) {
                                if (v.size() > 1) return set_err(err, ScriptError::MINIMALIF);
                                if (v.size() == 1 && v[0] != 1) return set_err(err, ScriptError::MINIMALIF);
                            }
                            value = cast_to_bool(v);
                            if (op == kOP_NOTIF) value = !value;
                            pop();
                        }
                        exec.push_back(value);
                        break;
                    }
                    case kOP_ELSE:
                        if (exec.empty()) return set_err(err, ScriptError::UNBALANCED_CONDITIONAL);
                        exec.back() = !exec.back();
                        break;
                    case kOP_ENDIF:
                        if (exec.empty()) return set_err(err, ScriptError::UNBALANCED_CONDITIONAL);
                        exec.pop_back();
                        break;
                    case kOP_VERIFY:
                        if (stack.size() < 1) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        if (!cast_to_bool(top(-1))) return set_err(err, ScriptError::VERIFY);
                        pop();
                        break;
                    case kOP_RETURN:
                        return set_err(err, ScriptError::OP_RETURN);
                    case kOP_TOALTSTACK:
                        if (stack.size() < 1) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        alt.push_back(top(-1));
                        pop();
                        break;
                    case kOP_FROMALTSTACK:
                        if (alt.size() < 1) return set_err(err, ScriptError::INVALID_ALTSTACK_OPERATION);
                        stack.push_back(alt.back());
                        alt.pop_back();
                        break;
                    case kOP_2DROP:
                        if (stack.size() < 2) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        pop();
                        pop();
                        break;
                    case kOP_2DUP: {
                        if (stack.size() < 2) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        Bytes a = top(-2), b = top(-1);
                        stack.push_back(a);
                        stack.push_back(b);
                        break;
                    }
                    case kOP_3DUP: {
                        if (stack.size() < 3) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        Bytes a = top(-3), b = top(-2), c = top(-1);
                        stack.push_back(a);
                        stack.push_back(b);
                        stack.push_back(c);
                        break;
                    }
                    case kOP_2OVER: {
                        if (stack.size() < 4) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        Bytes a = top(-4), b = top(-3);
                        stack.push_back(a);
                        stack.push_back(b);
                        break;
                    }
                    case kOP_2ROT: {
                        if (stack.size() < 6) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        Bytes a = top(-6), b = top(-5);
                        stack.erase(stack.end() - 6, stack.end() - 4);
                        stack.push_back(a);
                        stack.push_back(b);
                        break;
                    }
                    case kOP_2SWAP:
                        if (stack.size() < 4) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        std::swap(top(-4), top(-2));
                        std::swap(top(-3), top(-1));
                        break;
                    case kOP_IFDUP:
                        if (stack.size() < 1) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        if (cast_to_bool(top(-1))) stack.push_back(Bytes(top(-1)));
                        break;
                    case kOP_DEPTH:
                        stack.push_back(scriptnum_encode(int64_t(stack.size())));
                        break;
                    case kOP_DROP:
                        if (stack.size() < 1) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        pop();
                        break;
                    case kOP_DUP:
                        if (stack.size() < 1) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        stack.push_back(Bytes(top(-1)));
                        break;
                    case kOP_NIP:
                        if (stack.size() < 2) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        stack.erase(stack.end() - 2);
                        break;
                    case kOP_OVER:
                        if (stack.size() < 2) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        stack.push_back(Bytes(top(-2)));
                        break;
                    case kOP_PICK:
                    case kOP_ROLL: {
                        if (stack.size() < 2) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        const int n = scriptnum_getint(scriptnum_decode(top(-1), minimal));
                        pop();
                        if (n < 0 || size_t(n) >= stack.size()) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        Bytes v = top(-n - 1);
                        if (op == kOP_ROLL) stack.erase(stack.end() - n - 1);
                        stack.push_back(std::move(v));
                        break;
                    }
                    case kOP_ROT:
                        if (stack.size() < 3) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        std::swap(top(-3), top(-2));
                        std::swap(top(-2), top(-1));
                        break;
                    case kOP_SWAP:
                        if (stack.size() < 2) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        std::swap(top(-2), top(-1));
                        break;
                    case kOP_TUCK: {
                        if (stack.size() < 2) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        Bytes v = top(-1);
                        stack.insert(stack.end() - 2, std::move(v));
                        break;
                    }
                    case kOP_SIZE:
                        if (stack.size() < 1) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        stack.push_back(scriptnum_encode(int64_t(top(-1).size())));
                        break;
                    case kOP_EQUAL:
                    case kOP_EQUALVERIFY: {
                        if (stack.size() < 2) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        const bool eq = top(-2) == top(-1);
                        pop();
                        pop();
                        stack.push_back(eq ? kTrue : kFalse);
                        if (op == kOP_EQUALVERIFY) {
                            if (!eq) return set_err(err, ScriptError::EQUALVERIFY);
                            pop();
                        }
                        break;
                    }
                    case kOP_1ADD: case kOP_1SUB: case kOP_NEGATE: case kOP_ABS: case kOP_NOT: case kOP_0NOTEQUAL: {
                        if (stack.size() < 1) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        int64_t bn = scriptnum_decode(top(-1), minimal);
                        switch (op) {
                            case kOP_1ADD: bn += 1; break;
                            case kOP_1SUB: bn -= 1; break;
                            case kOP_NEGATE: bn = -bn; break;
                            case kOP_ABS: if (bn < 0) bn = -bn; break;
                            case kOP_NOT: bn = bn == 0; break;
                            default: bn = bn != 0; break;
                        }
                        pop();
                        stack.push_back(scriptnum_encode(bn));
                        break;
                    }
                    case kOP_ADD: case kOP_SUB: case kOP_BOOLAND: case kOP_BOOLOR: case kOP_NUMEQUAL:
                    case kOP_NUMEQUALVERIFY: case kOP_NUMNOTEQUAL: case kOP_LESSTHAN: case kOP_GREATERTHAN:
                    case kOP_LESSTHANOREQUAL: case kOP_GREATERTHANOREQUAL: case kOP_MIN: case kOP_MAX: {
                        if (stack.size() < 2) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        const int64_t a = scriptnum_decode(top(-2), minimal), b = scriptnum_decode(top(-1), minimal);
                        int64_t r = 0;
                        switch (op) {
                            case kOP_ADD: r = a + b; break;
                            case kOP_SUB: r = a - b; break;
                            case kOP_BOOLAND: r = a != 0 && b != 0; break;
                            case kOP_BOOLOR: r = a != 0 || b != 0; break;
                            case kOP_NUMEQUAL: case kOP_NUMEQUALVERIFY: r = a == b; break;
                            case kOP_NUMNOTEQUAL: r = a != b; break;
                            case kOP_LESSTHAN: r = a < b; break;
                            case kOP_GREATERTHAN: r = a > b; break;
                            case kOP_LESSTHANOREQUAL: r = a <= b; break;
                            case kOP_GREATERTHANOREQUAL: r = a >= b; break;
                            case kOP_MIN: r = a < b ? a : b; break;
                            default: r = a > b ? a : b; break;
                        }
                        pop();
                        pop();
                        stack.push_back(scriptnum_encode(r));
                        if (op == kOP_NUMEQUALVERIFY) {
                            if (!cast_to_bool(top(-1))) return set_err(err, ScriptError::NUMEQUALVERIFY);
                            pop();
                        }
                        break;
                    }
                    case kOP_WITHIN: {
                        if (stack.size() < 3) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        const int64_t x = scriptnum_decode(top(-3), minimal), lo = scriptnum_decode(top(-2), minimal),
                                      hi = scriptnum_decode(top(-1), minimal);
                        pop();
                        pop();
                        pop();
                        stack.push_back(lo <= x && x < hi ? kTrue : kFalse);
                        break;
                    }
                    case kOP_RIPEMD160: case kOP_SHA1: case kOP_SHA256: case kOP_HASH160: case kOP_HASH256: {
                        if (stack.size() < 1) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        const Bytes& v = top(-1);
                        Bytes h;
                        if (op == kOP_RIPEMD160) { h.resize(20); ripemd160(v.data(), v.size(), h.data()); }
                        else if (op == kOP_SHA1) { h.resize(20); sha1(v.data(), v.size(), h.data()); }
                        else if (op == kOP_SHA256) { h.resize(32); sha256(v.data(), v.size(), h.data()); }
                        else if (op == kOP_HASH160) { h.resize(20); hash160(v.data(), v.size(), h.data()); }
                        else { h.resize(32); sha256d(v.data(), v.size(), h.data()); }
                        pop();
                        stack.push_back(std::move(h));
                        break;
                    }
                    case kOP_CODESEPARATOR:
                        begin_code = pc;
                        break;
                    case kOP_CHECKSIG:
                    case kOP_CHECKSIGVERIFY: {
                        if (stack.size() < 2) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        const Bytes sig = top(-2), pk = top(-1);
                        Bytes code(script.begin() + begin_code, script.end());
                        if (sv == SigVersion::BASE) find_and_delete(code, push_script(sig));
                        if (!check_signature_encoding(sig, flags, err) || !check_pubkey_encoding(pk, flags, sv, err))
                            return false;
                        const bool ok = checker.check_sig(sig, pk, code, sv);
                        if (!ok && (flags & SCRIPT_VERIFY_NULLFAIL) && !sig.empty())
                            return set_err(err, ScriptError::NULLFAIL);
                        pop();
                        pop();
                        stack.push_back(ok ? kTrue : kFalse);
                        if (op == kOP_CHECKSIGVERIFY) {
                            if (!ok) return set_err(err, ScriptError::CHECKSIGVERIFY);
                            pop();
                        }
                        break;
                    }
                    case kOP_CHECKMULTISIG:
                    case kOP_CHECKMULTISIGVERIFY: {
                        int i = 1;
                        if ((int)stack.size() < i) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        int nkeys = scriptnum_getint(scriptnum_decode(top(-i), minimal));
                        if (nkeys < 0 || nkeys > kMaxPubkeysPerMultisig) return set_err(err, ScriptError::PUBKEY_COUNT);
                        op_count += nkeys;
                        if (op_count > kMaxOpsPerScript) return set_err(err, ScriptError::OP_COUNT);
                        int ikey = ++i;
                        int ikey2 = nkeys + 2;  // the keys' positions, for NULLFAIL
                        i += nkeys;
                        if ((int)stack.size() < i) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        int nsigs = scriptnum_getint(scriptnum_decode(top(-i), minimal));
                        if (nsigs < 0 || nsigs > nkeys) return set_err(err, ScriptError::SIG_COUNT);
                        int isig = ++i;
                        i += nsigs;
                        if ((int)stack.size() < i) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        Bytes code(script.begin() + begin_code, script.end());
                        for (int k = 0; k < nsigs; ++k) {
                            if (sv == SigVersion::BASE) find_and_delete(code, push_script(top(-isig - k)));
                        }
                        bool success = true;
                        while (success && nsigs > 0) {
                            const Bytes& sig = top(-isig);
                            const Bytes& pk = top(-ikey);
                            if (!check_signature_encoding(sig, flags, err) || !check_pubkey_encoding(pk, flags, sv, err))
                                return false;
                            if (checker.check_sig(sig, pk, code, sv)) {
                                ++isig;
                                --nsigs;
                            }
                            ++ikey;
                            --nkeys;
                            if (nsigs > nkeys) success = false;
                        }
                        while (i-- > 1) {
                            if (!success && (flags & SCRIPT_VERIFY_NULLFAIL) && !ikey2 && !top(-1).empty())
                                return set_err(err, ScriptError::NULLFAIL);
                            if (ikey2 > 0) --ikey2;
                            pop();
                        }
                        // the extra (dummy) element consumed by the historical off-by-one
                        if (stack.size() < 1) return set_err(err, ScriptError::INVALID_STACK_OPERATION);
                        if ((flags & SCRIPT_VERIFY_NULLDUMMY) && !top(-1).empty())
                            return set_err(err, ScriptError::SIG_NULLDUMMY);
                        pop();
                        stack.push_back(success ? kTrue : kFalse);
                        if (op == kOP_CHECKMULTISIGVERIFY) {
                            if (!success) return set_err(err, ScriptError::CHECKMULTISIGVERIFY);
                            pop();
                        }
                        break;
                    }
                    case OP_CLORE_ASSET:
                        break;  // asset payload: carried as data, no effect on evaluation
                    default:
                        return set_err(err, ScriptError::BAD_OPCODE);
                }
            }
            if (stack.size() + alt.size() > kMaxStackSize) return set_err(err, ScriptError::STACK_SIZE);
        }
    } catch (...) {
        return set_err(err, ScriptError::UNKNOWN_ERROR);
    }
    if (!exec.empty()) return set_err(err, ScriptError::UNBALANCED_CONDITIONAL);
    return set_err(err, ScriptError::OK);
}

namespace {

bool verify_witness_program(const std::vector<Bytes>& witness, int version, const Bytes& program, u32 flags,
                            const SigChecker& checker, ScriptError* err) {
    std::vector<Bytes> stack;
    Bytes spk;
    if (version == 0) {
        if (program.size() == 32) {
            if (witness.empty()) return set_err(err, ScriptError::WITNESS_PROGRAM_WITNESS_EMPTY);
            spk = witness.back();
            stack.assign(witness.begin(), witness.end() - 1);
            u8 h[32];
            sha256(spk.data(), spk.size(), h);
            if (std::memcmp(h, program.data(), 32) != 0) return set_err(err, ScriptError::WITNESS_PROGRAM_MISMATCH);
        } else if (program.size() == 20) {
            if (witness.size() != 2) return set_err(err, ScriptError::WITNESS_PROGRAM_MISMATCH);
            spk = {kOP_DUP, kOP_HASH160, 20};
            spk.insert(spk.end(), program.begin(), program.end());
            spk.push_back(kOP_EQUALVERIFY);
            spk.push_back(kOP_CHECKSIG);
            stack = witness;
        } else {
            return set_err(err, ScriptError::WITNESS_PROGRAM_WRONG_LENGTH);
        }
    } else if (flags & SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM) {
        return set_err(err, ScriptError::DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM);
    } else {
        return set_err(err, ScriptError::OK);  // future witness versions: anyone can spend
    }
    for (auto& e : stack)
        if (e.size() > kMaxScriptElementSize) return set_err(err, ScriptError::PUSH_SIZE);
    if (!eval_script(stack, spk, flags, checker, SigVersion::WITNESS_V0, err)) return false;
    if (stack.size() != 1) return set_err(err, ScriptError::EVAL_FALSE);
    if (!cast_to_bool(stack.back())) return set_err(err, ScriptError::EVAL_FALSE);
    return true;
}

}  // namespace

bool verify_script(const Bytes& script_sig, const Bytes& script_pubkey, const std::vector<Bytes>* witness, u32 flags,
                   const SigChecker& checker, ScriptError* err) {
    static const std::vector<Bytes> kEmpty;
    if (!witness) witness = &kEmpty;
    bool had_witness = false;
    set_err(err, ScriptError::UNKNOWN_ERROR);
    if ((flags & SCRIPT_VERIFY_SIGPUSHONLY) && !script_is_push_only(script_sig))
        return set_err(err, ScriptError::SIG_PUSHONLY);
    std::vector<Bytes> stack, copy;
    if (!eval_script(stack, script_sig, flags, checker, SigVersion::BASE, err)) return false;
    if (flags & SCRIPT_VERIFY_P2SH) copy = stack;
    if (!eval_script(stack, script_pubkey, flags, checker, SigVersion::BASE, err)) return false;
    if (stack.empty() || !cast_to_bool(stack.back())) return set_err(err, ScriptError::EVAL_FALSE);

    int version;
    Bytes program;
    if ((flags & SCRIPT_VERIFY_WITNESS) && script_is_witness_program(script_pubkey, version, program)) {
        had_witness = true;
        if (!script_sig.empty()) return set_err(err, ScriptError::WITNESS_MALLEATED);
        if (!verify_witness_program(*witness, version, program, flags, checker, err)) return false;
        stack.resize(1);  // bypass the cleanstack check below
    }
    if ((flags & SCRIPT_VERIFY_P2SH) && script_is_p2sh(script_pubkey)) {
        if (!script_is_push_only(script_sig)) return set_err(err, ScriptError::SIG_PUSHONLY);
        stack.swap(copy);
        const Bytes redeem = stack.back();
        stack.pop_back();
        if (!eval_script(stack, redeem, flags, checker, SigVersion::BASE, err)) return false;
        if (stack.empty() || !cast_to_bool(stack.back())) return set_err(err, ScriptError::EVAL_FALSE);
        if ((flags & SCRIPT_VERIFY_WITNESS) && script_is_witness_program(redeem, version, program)) {
            had_witness = true;
            if (script_sig != push_script(redeem)) return set_err(err, ScriptError::WITNESS_MALLEATED_P2SH);
            if (!verify_witness_program(*witness, version, program, flags, checker, err)) return false;
            stack.resize(1);
        }
    }
    if (flags & SCRIPT_VERIFY_CLEANSTACK) {
        if (stack.size() != 1) return set_err(err, ScriptError::CLEANSTACK);
    }
    if (flags & SCRIPT_VERIFY_WITNESS) {
        if (!had_witness && !witness->empty()) return set_err(err, ScriptError::WITNESS_UNEXPECTED);
    }
    return set_err(err, ScriptError::OK);
}

std::string check_transaction(const Transaction& tx, bool check_duplicate_inputs, const assets::Params* asset_params,
                              const assets::Flags* flags, bool block_check, bool mempool_check) {
    if (tx.vin.empty()) return "bad-txns-vin-empty";
    if (tx.vout.empty()) return "bad-txns-vout-empty";
    if (tx.bytes(false).size() * 4 > 8000000) return "bad-txns-oversize";  // GetMaxBlockWeight() after HIP2
    Amount out = 0;
    for (auto& o : tx.vout) {
        if (o.value < 0) return "bad-txns-vout-negative";
        if (o.value > kMaxMoney) return "bad-txns-vout-toolarge";
        out += o.value;
        if (out < 0 || out > kMaxMoney) return "bad-txns-txouttotal-toolarge";
    }
    if (check_duplicate_inputs) {
        std::set<std::pair<Uint256, u32>> seen;
        for (auto& in : tx.vin)
            if (!seen.insert({in.prevout.hash, in.prevout.n}).second) return "bad-txns-inputs-duplicate";
    }
    if (tx.is_coinbase()) {
        if (tx.vin[0].script_sig.size() < 2 || tx.vin[0].script_sig.size() > 100) return "bad-cb-length";
    } else {
        for (auto& in : tx.vin)
            if (in.prevout.is_null()) return "bad-txns-prevout-null";
    }
    if (asset_params) {
        const assets::Flags none;
        return assets::check_tx_structure(tx, *asset_params, flags ? *flags : none, block_check, mempool_check);
    }
    return "";
}

}  // namespace nodexa
