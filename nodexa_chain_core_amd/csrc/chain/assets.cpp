// Asset layer: see assets.hpp.
#include "assets.hpp"

#include <algorithm>
#include <cctype>
#include <stdexcept>

#include "coins.hpp"
#include "interpreter.hpp"
#include "script.hpp"
#include "serialize.hpp"

namespace nodexa::assets {

// ------------------------------------------------------------------ names
namespace {

bool all_of_set(const std::string& s, bool (*ok)(char)) {
    return std::all_of(s.begin(), s.end(), [&](char c) { return ok(c); });
}
bool upper_digit_dot_us(char c) { return (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '.' || c == '_'; }
bool unique_tag_char(char c) {
    if (std::isalnum(static_cast<unsigned char>(c))) return true;
    static const std::string extra = "-@$%&*()[]{}_.?:";
    return extra.find(c) != std::string::npos;
}
bool channel_char(char c) { return std::isalnum(static_cast<unsigned char>(c)) || c == '_'; }
bool punct(char c) { return c == '.' || c == '_'; }

bool double_punct(const std::string& s) {
    for (size_t i = 1; i < s.size(); ++i)
        if (punct(s[i]) && punct(s[i - 1])) return true;
    return false;
}
bool lead_punct(const std::string& s) { return !s.empty() && punct(s.front()); }
bool trail_punct(const std::string& s) { return !s.empty() && punct(s.back()); }
bool reserved(const std::string& s) {
    static const char* names[] = {"RVN", "RAVEN", "RAVENCOIN", "#RVN", "#RAVEN", "#RAVENCOIN",
                                  "CLORE", "CLORECOIN", "#CLORE", "#CLORECOIN"};
    for (auto* n : names)
        if (s == n) return true;
    return false;
}
bool clean(const std::string& s) { return !double_punct(s) && !lead_punct(s) && !trail_punct(s); }

bool root_ok(const std::string& s) {
    return s.size() >= 3 && all_of_set(s, upper_digit_dot_us) && clean(s) && !reserved(s);
}
bool sub_ok(const std::string& s) { return !s.empty() && all_of_set(s, upper_digit_dot_us) && clean(s); }
// '#' or '$' followed by at least `min` name characters
bool tagged_ok(const std::string& s, char lead, size_t min) {
    return s.size() >= 1 + min && s[0] == lead && all_of_set(s.substr(1), upper_digit_dot_us);
}
bool qualifier_ok(const std::string& s) {
    return tagged_ok(s, '#', 3) && !double_punct(s) && !(s.size() > 1 && punct(s[1])) && !trail_punct(s) &&
           !reserved(s);
}
bool sub_qualifier_ok(const std::string& s) { return tagged_ok(s, '#', 1) && clean(s); }
bool restricted_ok(const std::string& s) { return tagged_ok(s, '$', 3) && clean(s) && !reserved(s); }

std::vector<std::string> split(const std::string& s, char d) {
    std::vector<std::string> out(1);
    for (char c : s) {
        if (c == d) out.emplace_back();
        else out.back() += c;
    }
    return out;
}

bool name_before_tag_ok(const std::string& name) {
    auto parts = split(name, '/');
    if (!root_ok(parts[0])) return false;
    for (size_t i = 1; i < parts.size(); ++i)
        if (!sub_ok(parts[i])) return false;
    return true;
}
bool qualifier_before_tag_ok(const std::string& name) {
    auto parts = split(name, '/');
    if (!qualifier_ok(parts[0]) || parts.size() > 2) return false;
    return parts.size() == 1 || sub_qualifier_ok(parts[1]);
}
bool is_subasset(const std::string& name) {
    auto parts = split(name, '/');
    return root_ok(parts[0]) && parts.size() > 1;
}
bool is_subqualifier(const std::string& name) {
    auto parts = split(name, '/');
    return qualifier_ok(parts[0]) && parts.size() > 1;
}

bool has_any(const std::string& s, const char* chars) { return s.find_first_of(chars) != std::string::npos; }
// "<prefix><delim><suffix>": prefix without ^~#!, suffix without ~#!/ (UNIQUE / MSGCHANNEL / VOTE indicators)
bool tag_indicator(const std::string& s, char delim) {
    const size_t at = s.find(delim);
    if (at == std::string::npos || at == 0 || at + 1 >= s.size()) return false;
    const std::string pre = s.substr(0, at), post = s.substr(at + 1);
    return !has_any(pre, "^~#!") && !has_any(post, "~#!/");
}
bool owner_indicator(const std::string& s) {
    return s.size() >= 2 && s.back() == '!' && !has_any(s.substr(0, s.size() - 1), "^~#!");
}
bool qualifier_indicator(const std::string& s) { return tagged_ok(s, '#', 3); }
bool sub_qualifier_indicator(const std::string& s) {
    const size_t at = s.find('/');
    if (at == std::string::npos) return false;
    return tagged_ok(s.substr(0, at), '#', 1) && tagged_ok(s.substr(at + 1), '#', 1);
}
bool restricted_indicator(const std::string& s) { return tagged_ok(s, '$', 3); }

constexpr size_t kMaxNameLength = 31;
constexpr size_t kMaxChannelLength = 12;

bool type_check(Type t, const std::string& name, std::string* err) {
    auto fail = [&](const std::string& e) {
        if (err) *err = e;
        return false;
    };
    const std::string too_long = "Name is greater than max length of " + std::to_string(kMaxNameLength);
    switch (t) {
        case Type::UNIQUE: {
            if (name.size() > kMaxNameLength) return fail(too_long);
            auto parts = split(name, '#');
            if (!(name_before_tag_ok(parts.front()) && !parts.back().empty() && all_of_set(parts.back(), unique_tag_char)))
                return fail("Unique name contains invalid characters");
            return true;
        }
        case Type::MSGCHANNEL: {
            if (name.size() > kMaxNameLength) return fail(too_long);
            auto parts = split(name, '~');
            const std::string& tag = parts.back();
            const bool ok = name_before_tag_ok(parts.front()) && !tag.empty() && all_of_set(tag, channel_char) && clean(tag);
            if (tag.size() > kMaxChannelLength)
                return fail("Channel name is greater than max length of " + std::to_string(kMaxChannelLength));
            if (!ok) return fail("Message Channel name contains invalid characters");
            return true;
        }
        case Type::OWNER:
            if (name.size() > kMaxNameLength) return fail(too_long);
            if (!name_before_tag_ok(name.substr(0, name.size() - 1))) return fail("Owner name contains invalid characters");
            return true;
        case Type::VOTE: {
            if (name.size() > kMaxNameLength) return fail(too_long);
            auto parts = split(name, '^');
            if (!(name_before_tag_ok(parts.front()) && !parts.back().empty() && all_of_set(parts.back(), upper_digit_dot_us)))
                return fail("Vote name contains invalid characters");
            return true;
        }
        case Type::QUALIFIER:
        case Type::SUB_QUALIFIER:
            if (name.size() > kMaxNameLength) return fail(too_long);
            if (!qualifier_before_tag_ok(name)) return fail("Qualifier name contains invalid characters");
            return true;
        case Type::RESTRICTED:
            if (name.size() > kMaxNameLength) return fail(too_long);
            if (!restricted_ok(name)) return fail("Restricted name contains invalid characters");
            return true;
        default: {
            if (name.size() > kMaxNameLength - 1)
                return fail("Name is greater than max length of " + std::to_string(kMaxNameLength - 1));
            if (!is_subasset(name) && name.size() < 3) return fail("Name must be contain 3 characters");
            if (!name_before_tag_ok(name)) return fail("Name contains invalid characters");
            return true;
        }
    }
}

}  // namespace

const char* type_name(Type t) {
    switch (t) {
        case Type::ROOT: return "ROOT";
        case Type::SUB: return "SUB";
        case Type::UNIQUE: return "UNIQUE";
        case Type::MSGCHANNEL: return "MSGCHANNEL";
        case Type::OWNER: return "OWNER";
        case Type::VOTE: return "VOTE";
        case Type::REISSUE: return "REISSUE";
        case Type::QUALIFIER: return "QUALIFIER";
        case Type::SUB_QUALIFIER: return "SUB_QUALIFIER";
        case Type::RESTRICTED: return "RESTRICTED";
        case Type::NULL_ADD_QUALIFIER: return "NULL_ADD_QUALIFIER";
        default: return "INVALID";
    }
}

Type name_type(const std::string& name, std::string* err) {
    if (name.size() > 40) return Type::INVALID;
    Type t;
    if (tag_indicator(name, '#') && !name.empty() && name[0] != '#') t = Type::UNIQUE;
    else if (tag_indicator(name, '~')) t = Type::MSGCHANNEL;
    else if (owner_indicator(name)) t = Type::OWNER;
    else if (tag_indicator(name, '^')) t = Type::VOTE;
    else if (qualifier_indicator(name)) t = Type::QUALIFIER;
    else if (sub_qualifier_indicator(name)) t = Type::SUB_QUALIFIER;
    else if (restricted_indicator(name)) t = Type::RESTRICTED;
    else t = is_subasset(name) ? Type::SUB : Type::ROOT;
    if (!type_check(t, name, err)) return Type::INVALID;
    if (t == Type::QUALIFIER && is_subqualifier(name)) t = Type::SUB_QUALIFIER;
    return t;
}

std::string parent_name(const std::string& name) {
    const Type t = name_type(name);
    char delim = 0;
    switch (t) {
        case Type::INVALID: return "";
        case Type::SUB:
        case Type::SUB_QUALIFIER: delim = '/'; break;
        case Type::UNIQUE: delim = '#'; break;
        case Type::MSGCHANNEL: delim = '~'; break;
        case Type::VOTE: delim = '^'; break;
        default: return name;
    }
    const size_t at = name.find_last_of(delim);
    return at == std::string::npos ? name : name.substr(0, at);
}

bool is_owner_name(const std::string& name) { return name_type(name) == Type::OWNER; }

bool amount_fits_units(int64_t amount, int units) {
    if (units < 0 || units > kMaxUnit) return false;
    int64_t m = 1;
    for (int i = 0; i < kMaxUnit - units; ++i) m *= 10;
    return amount % m == 0;
}

// ------------------------------------------------------------------ verifier expressions
namespace {

bool name_char(char c) { return std::isalnum(static_cast<unsigned char>(c)) || c == '_' || c == '#' || c == '.'; }

// Top-level pieces of `f` separated by `op` (parenthesised groups stay whole; operators before
// the first piece are skipped; an operator that is neither & nor | is an error).
std::vector<std::string> pieces(const std::string& f, char op) {
    std::vector<std::string> out;
    int depth = 0;
    long start = -1;
    for (size_t i = 0; i < f.size(); ++i) {
        const char c = f[i];
        if (c == ')') {
            --depth;
        } else if (c == '(') {
            if (depth++ == 0 && start < 0) start = long(i);
        } else if (depth == 0) {
            const bool part = name_char(c) || c == '!';
            if (start < 0) {
                if (part) start = long(i);
            } else if (!part) {
                if (c == op) {
                    out.push_back(f.substr(size_t(start), i - size_t(start)));
                    start = long(i) + 1;
                } else if (c != '&' && c != '|') {
                    throw std::runtime_error("Unknown operator '" + std::string(1, c) + "' in the (sub)expression '" + f + "'.");
                }
            }
        }
    }
    if (start >= 0) out.push_back(f.substr(size_t(start)));
    if (depth != 0) throw std::runtime_error("Wrong parenthesis parity in the (sub)expression '" + f + "'.");
    return out;
}

bool eval(const std::string& f, const std::map<std::string, bool>& vals) {
    if (f.empty()) throw std::runtime_error("An empty subexpression was encountered");
    char op = '|';
    auto parts = pieces(f, op);
    if (parts.size() == 1) {
        op = '&';
        parts = pieces(f, op);
    }
    if (parts.empty()) throw std::runtime_error("The subexpression " + f + " is not a valid formula.");
    if (parts.size() == 1) {
        if (f[0] == '!') return !eval(f.substr(1), vals);
        if (f[0] == '(') return eval(f.substr(1, f.size() - 2), vals);
        if (f == "1") return true;
        if (f == "0") return false;
        auto it = vals.find(f);
        if (it == vals.end()) throw std::runtime_error("Variable '" + f + "' not found in the interpretation.");
        return it->second;
    }
    bool acc = op == '&';
    for (auto& p : parts) {
        const bool v = eval(p, vals);  // every piece is evaluated (errors surface as in the reference)
        acc = op == '&' ? (acc && v) : (acc || v);
    }
    return acc;
}

std::string no_space(const std::string& s) {
    std::string r;
    for (char c : s)
        if (!std::isspace(static_cast<unsigned char>(c))) r += c;
    return r;
}

}  // namespace

bool bool_expr(const std::string& expr, const std::map<std::string, bool>& vals) { return eval(no_space(expr), vals); }

std::string strip_verifier(const std::string& v) {
    std::string r;
    for (char c : no_space(v))
        if (c != '#') r += c;
    return r;
}

std::set<std::string> verifier_qualifiers(const std::string& s) {
    std::set<std::string> out;
    std::string cur;
    for (char c : s) {
        if (upper_digit_dot_us(c)) {
            cur += c;
        } else if (!cur.empty()) {
            out.insert(cur);
            cur.clear();
        }
    }
    if (!cur.empty()) out.insert(cur);
    return out;
}

bool check_verifier(const std::string& verifier, std::set<std::string>& found, std::string& err) {
    if (verifier == "true") return true;
    if (verifier.empty()) {
        err = "Verifier string can not be empty. To default to true, use \"true\"";
        return false;
    }
    const std::string stripped = strip_verifier(verifier);
    if (stripped.size() > 80) {
        err = "Verifier string has length greater than 80 after whitespaces and '#' are removed";
        return false;
    }
    found = verifier_qualifiers(stripped);
    std::map<std::string, bool> vals;
    for (auto& q : found) {
        if (!qualifier_ok("#" + q)) {
            err = "bad-txns-null-verifier-invalid-asset-name-" + q;
            return false;
        }
        vals[q] = true;
    }
    try {
        bool_expr(verifier, vals);
    } catch (const std::runtime_error&) {
        err = "bad-txns-null-verifier-failed-syntax-check";
        return false;
    }
    return true;
}

// ------------------------------------------------------------------ scripts
namespace {

std::string read_str(Reader& r) {
    const Bytes b = r.var_bytes();
    return std::string(b.begin(), b.end());
}
void write_str(Writer& w, const std::string& s) { w.var_bytes(Bytes(s.begin(), s.end())); }

// ReadWriteAssetHash (read side): 34-byte multihash (prefix kept) or the 32 bytes after another marker
bool read_hash(Reader& r, std::string& out) {
    out.clear();
    if (r.remaining() < 33) return false;
    const u8 marker = r.u8_();
    const std::string h = read_str(r);
    if (marker == 0x12) out = std::string("\x12\x20", 2);
    out += h.substr(0, 32);
    return true;
}
bool write_hash(Writer& w, const std::string& h) {
    if (h.size() == 34) {
        w.u8_(0x12);
        write_str(w, h.substr(2));
        return true;
    }
    if (h.size() == 32) {
        w.u8_(0x54);  // TXID_NOTIFIER
        write_str(w, h);
        return true;
    }
    return false;
}

Bytes push(const Bytes& d) {
    Bytes s;
    if (d.size() < OP_PUSHDATA1) {
        s.push_back(u8(d.size()));
    } else if (d.size() <= 0xff) {
        s.push_back(OP_PUSHDATA1);
        s.push_back(u8(d.size()));
    } else {
        s.push_back(OP_PUSHDATA2);
        s.push_back(u8(d.size() & 0xff));
        s.push_back(u8(d.size() >> 8));
    }
    s.insert(s.end(), d.begin(), d.end());
    return s;
}

Bytes p2pkh(const u8 h160[20]) {
    Bytes s = {OP_DUP, OP_HASH160, 20};
    s.insert(s.end(), h160, h160 + 20);
    s.push_back(OP_EQUALVERIFY);
    s.push_back(OP_CHECKSIG);
    return s;
}

Bytes asset_script(const u8 h160[20], char kind, const Bytes& payload) {
    Bytes msg = {'r', 'v', 'n', u8(kind)};
    msg.insert(msg.end(), payload.begin(), payload.end());
    Bytes s = p2pkh(h160);
    s.push_back(kOpAsset);
    const Bytes p = push(msg);
    s.insert(s.end(), p.begin(), p.end());
    s.push_back(0x75);  // OP_DROP
    return s;
}

}  // namespace

OutKind asset_script_kind(const Bytes& s, size_t* payload_at) {
    if (s.size() <= 31 || s[25] != kOpAsset) return OutKind::NONE;
    int index = -1;
    if (s[27] == 'r') {
        if (s[28] == 'v' && s[29] == 'n') index = 30;
    } else if (s[28] == 'r' && s[29] == 'v' && s[30] == 'n') {
        index = 31;
    }
    if (index < 0) return OutKind::NONE;
    OutKind k = OutKind::NONE;
    switch (s[size_t(index)]) {
        case 't': k = OutKind::TRANSFER; break;
        case 'q': k = s.size() > 39 ? OutKind::NEW : OutKind::NONE; break;
        case 'o': k = OutKind::OWNER; break;
        case 'r': k = OutKind::REISSUE; break;
        default: break;
    }
    if (k != OutKind::NONE && payload_at) *payload_at = size_t(index) + 1;
    return k;
}

bool parse_asset_out(const Bytes& spk, AssetOut& a) {
    size_t at = 0;
    a = AssetOut{};
    const OutKind k = asset_script_kind(spk, &at);
    if (k == OutKind::NONE) return false;
    a.kind = k;
    std::memcpy(a.h160, spk.data() + 3, 20);
    try {
        Reader r(spk.data() + at, spk.size() - at);
        switch (k) {
            case OutKind::NEW:
                a.name = read_str(r);
                a.amount = r.i64_();
                a.units = int8_t(r.u8_());
                a.reissuable = int8_t(r.u8_());
                a.has_ipfs = int8_t(r.u8_());
                if (a.has_ipfs == 1) read_hash(r, a.ipfs);
                break;
            case OutKind::OWNER:
                a.name = read_str(r);
                a.amount = kOwnerAmount;
                break;
            case OutKind::TRANSFER:
                a.name = read_str(r);
                a.amount = r.i64_();
                if (read_hash(r, a.message) && r.remaining() >= 8) a.expire = r.i64_();
                break;
            case OutKind::REISSUE:
                a.name = read_str(r);
                a.amount = r.i64_();
                a.units = int8_t(r.u8_());
                a.reissuable = int8_t(r.u8_());
                read_hash(r, a.ipfs);
                break;
            default: return false;
        }
    } catch (const std::exception&) {
        return false;
    }
    return true;
}

bool asset_amount(const Bytes& spk, int64_t& amount) {
    AssetOut a;
    if (!parse_asset_out(spk, a)) return false;
    amount = a.amount;
    return true;
}

bool script_unspendable(const Bytes& spk) {
    if (!spk.empty() && (spk[0] == OP_RETURN || spk[0] == kOpAsset)) return true;
    if (spk.size() > kMaxScriptSize) return true;
    int64_t amount;
    return asset_amount(spk, amount) && amount == 0;
}

NullKind null_kind(const Bytes& s) {
    if (s.size() > 23 && s[0] == kOpAsset && s[1] == 0x14) return NullKind::TAG;
    if (s.size() > 6 && s[0] == kOpAsset && s[1] == 0x50 && s[2] == 0x50) return NullKind::GLOBAL;
    if (s.size() > 3 && s[0] == kOpAsset && s[1] == 0x50 && s[2] != 0x50) return NullKind::VERIFIER;
    return NullKind::NONE;
}

bool parse_null_tag(const Bytes& s, std::string& name, int& flag, u8 h160[20]) {
    if (null_kind(s) != NullKind::TAG) return false;
    std::memcpy(h160, s.data() + 2, 20);
    try {
        Reader r(s.data() + 23, s.size() - 23);
        name = read_str(r);
        flag = int8_t(r.u8_());
    } catch (const std::exception&) {
        return false;
    }
    return true;
}

bool parse_null_global(const Bytes& s, std::string& name, int& flag) {
    if (null_kind(s) != NullKind::GLOBAL) return false;
    try {
        Reader r(s.data() + 4, s.size() - 4);
        name = read_str(r);
        flag = int8_t(r.u8_());
    } catch (const std::exception&) {
        return false;
    }
    return true;
}

bool parse_null_verifier(const Bytes& s, std::string& verifier) {
    if (null_kind(s) != NullKind::VERIFIER) return false;
    try {
        Reader r(s.data() + 3, s.size() - 3);
        verifier = read_str(r);
    } catch (const std::exception&) {
        return false;
    }
    return true;
}

Bytes script_new(const u8 h160[20], const AssetOut& a) {
    Writer w;
    write_str(w, a.name);
    w.i64_(a.amount);
    w.u8_(u8(int8_t(a.units)));
    w.u8_(u8(int8_t(a.reissuable)));
    w.u8_(u8(int8_t(a.has_ipfs)));
    if (a.has_ipfs == 1) write_hash(w, a.ipfs);
    return asset_script(h160, 'q', w.buf);
}

Bytes script_owner(const u8 h160[20], const std::string& name) {
    Writer w;
    write_str(w, name);
    return asset_script(h160, 'o', w.buf);
}

Bytes script_transfer(const u8 h160[20], const std::string& name, int64_t amount, const std::string& message,
                      int64_t expire) {
    Writer w;
    write_str(w, name);
    w.i64_(amount);
    if (write_hash(w, message) && expire != 0) w.i64_(expire);
    return asset_script(h160, 't', w.buf);
}

Bytes script_reissue(const u8 h160[20], const std::string& name, int64_t amount, int units, int reissuable,
                     const std::string& ipfs) {
    Writer w;
    write_str(w, name);
    w.i64_(amount);
    w.u8_(u8(int8_t(units)));
    w.u8_(u8(int8_t(reissuable)));
    write_hash(w, ipfs);
    return asset_script(h160, 'r', w.buf);
}

Bytes script_null_tag(const u8 h160[20], const std::string& name, int flag) {
    Writer w;
    write_str(w, name);
    w.u8_(u8(int8_t(flag)));
    Bytes s = {kOpAsset, 20};
    s.insert(s.end(), h160, h160 + 20);
    const Bytes p = push(w.buf);
    s.insert(s.end(), p.begin(), p.end());
    return s;
}

Bytes script_null_global(const std::string& name, int flag) {
    Writer w;
    write_str(w, name);
    w.u8_(u8(int8_t(flag)));
    Bytes s = {kOpAsset, 0x50, 0x50};
    const Bytes p = push(w.buf);
    s.insert(s.end(), p.begin(), p.end());
    return s;
}

Bytes script_null_verifier(const std::string& verifier) {
    Writer w;
    write_str(w, verifier);
    Bytes s = {kOpAsset, 0x50};
    const Bytes p = push(w.buf);
    s.insert(s.end(), p.begin(), p.end());
    return s;
}

// ------------------------------------------------------------------ params
int64_t Params::burn_amount(Type t) const {
    switch (t) {
        case Type::ROOT: return burn_root;
        case Type::SUB: return burn_sub;
        case Type::UNIQUE: return burn_unique;
        case Type::MSGCHANNEL: return burn_msgchannel;
        case Type::QUALIFIER: return burn_qualifier;
        case Type::SUB_QUALIFIER: return burn_subqualifier;
        case Type::RESTRICTED: return burn_restricted;
        case Type::NULL_ADD_QUALIFIER: return burn_tag;
        default: return 0;
    }
}

const Bytes* Params::burn_script(Type t) const {
    switch (t) {
        case Type::ROOT: return &spk_root;
        case Type::SUB: return &spk_sub;
        case Type::UNIQUE: return &spk_unique;
        case Type::MSGCHANNEL: return &spk_msgchannel;
        case Type::QUALIFIER: return &spk_qualifier;
        case Type::SUB_QUALIFIER: return &spk_subqualifier;
        case Type::RESTRICTED: return &spk_restricted;
        case Type::NULL_ADD_QUALIFIER: return &spk_tag;
        default: return nullptr;
    }
}

// ------------------------------------------------------------------ transaction classification
namespace {

// the name type of a new-asset ('q') output, INVALID if it is none or does not parse
Type new_out_type(const TxOut& o, AssetOut* a = nullptr) {
    AssetOut tmp;
    AssetOut& x = a ? *a : tmp;
    if (asset_script_kind(o.script_pubkey) != OutKind::NEW || !parse_asset_out(o.script_pubkey, x)) return Type::INVALID;
    return name_type(x.name);
}

bool burn_found(const Transaction& tx, const Params& p, Type t, int n = 1) {
    if (t == Type::REISSUE || t == Type::VOTE || t == Type::OWNER || t == Type::INVALID) return false;
    const Bytes* spk = p.burn_script(t);
    const int64_t amount = p.burn_amount(t) * n;
    for (auto& o : tx.vout)
        if (o.value == amount && spk && !spk->empty() && o.script_pubkey == *spk) return true;
    return false;
}

bool reissue_burn_found(const Transaction& tx, const Params& p) {
    for (auto& o : tx.vout)
        if (o.value == p.burn_reissue && !p.spk_reissue.empty() && o.script_pubkey == p.spk_reissue) return true;
    return false;
}

bool transfer_of(const Transaction& tx, const std::string& name) {
    for (auto& o : tx.vout) {
        AssetOut a;
        if (asset_script_kind(o.script_pubkey) == OutKind::TRANSFER && parse_asset_out(o.script_pubkey, a) &&
            a.name == name)
            return true;
    }
    return false;
}

struct Counts {
    int issues = 0, reissues = 0, transfers = 0, owners = 0;
};
Counts count_kinds(const Transaction& tx) {
    Counts c;
    for (auto& o : tx.vout) {
        switch (asset_script_kind(o.script_pubkey)) {
            case OutKind::NEW: ++c.issues; break;
            case OutKind::OWNER: ++c.owners; break;
            case OutKind::TRANSFER: ++c.transfers; break;
            case OutKind::REISSUE: ++c.reissues; break;
            default: break;
        }
    }
    return c;
}

// GetVerifierStringFromTx: 1 = found, 0 = none, -1 = malformed or more than one
int tx_verifier(const Transaction& tx, std::string& v) {
    int n = 0;
    for (auto& o : tx.vout) {
        if (null_kind(o.script_pubkey) != NullKind::VERIFIER) continue;
        if (++n > 1) return -1;
        if (!parse_null_verifier(o.script_pubkey, v)) return -1;
    }
    return n;
}

bool find_op(const Bytes& s, u8 op) {
    size_t pc = 0;
    u8 o;
    while (pc < s.size()) {
        if (!script_get_op(s, pc, o, nullptr)) return false;
        if (o == op) return true;
    }
    return false;
}

const int64_t kMaxMoneyAssets = 21000000000LL * kCoin;  // MAX_MONEY of the asset amount checks

std::string check_new_asset(const AssetOut& a) {
    const Type t = name_type(a.name);
    const std::string prefix = "Invalid parameter: ";
    if (t == Type::INVALID) return prefix + "asset_name must only consist of valid characters";
    if (t == Type::UNIQUE || t == Type::MSGCHANNEL) {
        if (a.units != 0) return prefix + "units must be 0";
        if (a.amount != kUniqueAmount) return prefix + "amount must be 100000000";
        if (a.reissuable != 0) return prefix + "reissuable must be 0";
    }
    if (t == Type::QUALIFIER || t == Type::SUB_QUALIFIER) {
        if (a.units != 0) return prefix + "units must be 0";
        if (a.amount < kQualifierMin || a.amount > kQualifierMax) return prefix + "amount must be between 1 - 10";
        if (a.reissuable != 0) return prefix + "reissuable must be 0";
    }
    if (t == Type::OWNER) return "Invalid parameters: asset_name can't have a '!' at the end of it";
    if (a.amount <= 0) return prefix + "asset amount can't be equal to or less than zero.";
    if (a.amount > kMaxMoneyAssets) return prefix + "asset amount greater than max money";
    if (a.units < 0 || a.units > 8) return prefix + "units must be between 0-8.";
    if (!amount_fits_units(a.amount, a.units)) return prefix + "amount must be divisible by the smaller unit assigned to the asset";
    if (a.reissuable != 0 && a.reissuable != 1) return prefix + "reissuable must be 0 or 1";
    if (a.has_ipfs != 0 && a.has_ipfs != 1) return prefix + "has_ipfs must be 0 or 1.";
    return "";
}

std::string check_reissue(const AssetOut& a, bool testnet) {
    if (a.amount < 0 || a.amount >= kMaxMoneyAssets) return "Unable to reissue asset: amount must be 0 or larger";
    if (a.units > kMaxUnit || a.units < -1) return "Unable to reissue asset: unit must be between 8 and -1";
    const bool skip = testnet && ((a.name == "GAMINGWEB" && a.reissuable == 109) || (a.name == "UINT8" && a.reissuable == -47));
    if (!skip && a.reissuable != 0 && a.reissuable != 1) return "Unable to reissue asset: reissuable must be 0 or 1";
    return "";
}

}  // namespace

TxKind tx_kind(const Transaction& tx) {
    if (tx.vout.empty()) return TxKind::NONE;
    const TxOut& last = tx.vout.back();
    const bool last_new = asset_script_kind(last.script_pubkey) == OutKind::NEW;
    if (last_new && tx.vout.size() >= 3 &&
        asset_script_kind(tx.vout[tx.vout.size() - 2].script_pubkey) == OutKind::OWNER) {
        const Type t = new_out_type(last);
        if (t != Type::UNIQUE && t != Type::RESTRICTED) return TxKind::NEW;
    }
    if (asset_script_kind(last.script_pubkey) == OutKind::REISSUE) return TxKind::REISSUE;
    if (!last_new) return TxKind::NONE;
    switch (new_out_type(last)) {
        case Type::UNIQUE: return TxKind::NEW_UNIQUE;
        case Type::MSGCHANNEL: return TxKind::NEW_MSGCHANNEL;
        case Type::QUALIFIER:
        case Type::SUB_QUALIFIER: return TxKind::NEW_QUALIFIER;
        case Type::RESTRICTED: return TxKind::NEW_RESTRICTED;
        default: return TxKind::NONE;
    }
}

std::string check_tx_structure(const Transaction& tx, const Params& p, const Flags& f, bool block_check,
                               bool mempool_check) {
    std::set<std::string> transfer_names;
    std::map<std::pair<std::string, std::string>, int> tag_count;
    std::set<std::string> global_changes;
    bool has_verifier = false;
    int add_tags = 0;
    for (auto& o : tx.vout) {
        switch (null_kind(o.script_pubkey)) {
            case NullKind::TAG: {
                std::string name;
                int flag;
                u8 h[20];
                if (!parse_null_tag(o.script_pubkey, name, flag, h)) return "bad-txns-null-asset-data-serialization";
                if (flag != 0 && flag != 1) return "bad-txns-null-data-flag-must-be-0-or-1";
                if (++tag_count[{name, std::string(reinterpret_cast<char*>(h), 20)}] > 1)
                    return "bad-txns-null-data-only-one-change-per-asset-address";
                const Type t = name_type(name);
                if ((t == Type::QUALIFIER || t == Type::SUB_QUALIFIER) && flag == 1) ++add_tags;
                break;
            }
            case NullKind::GLOBAL: {
                std::string name;
                int flag;
                if (!parse_null_global(o.script_pubkey, name, flag)) return "bad-txns-null-global-asset-data-serialization";
                if (flag != 0 && flag != 1) return "bad-txns-null-data-flag-must-be-0-or-1";
                if (!global_changes.insert(name).second) return "bad-txns-null-data-only-one-global-change-per-asset-name";
                break;
            }
            case NullKind::VERIFIER: {
                std::string v;
                if (!parse_null_verifier(o.script_pubkey, v)) return "bad-txns-null-verifier-data-serialization";
                if (v.find(' ') != std::string::npos) return "bad-txns-null-verifier-data-contained-whitespaces";
                if (v.find('#') != std::string::npos) return "bad-txns-null-verifier-data-contained-qualifier-character-#";
                std::set<std::string> found;
                std::string err;
                if (!check_verifier(v, found, err)) return err;
                if (has_verifier) return "bad-txns-null-data-only-one-verifier-per-tx";
                has_verifier = true;
                break;
            }
            default: break;
        }
        const OutKind k = asset_script_kind(o.script_pubkey);
        if (k == OutKind::TRANSFER) {
            AssetOut a;
            if (!parse_asset_out(o.script_pubkey, a)) return "bad-txns-transfer-asset-bad-deserialize";
            transfer_names.insert(a.name);
            const Type t = name_type(a.name);
            if (t == Type::INVALID) return "bad-txns-transfer-asset-name-invalid";
            if (t == Type::OWNER && a.amount != kOwnerAmount) return "bad-txns-transfer-owner-amount-was-not-1";
            if (t == Type::UNIQUE && a.amount != kUniqueAmount) return "bad-txns-transfer-unique-amount-was-not-1";
            if ((t == Type::QUALIFIER || t == Type::SUB_QUALIFIER) && (a.amount < kQualifierMin || a.amount > kQualifierMax))
                return "bad-txns-transfer-qualifier-amount-must be between 1 - 100";
            if (o.value != 0) return "bad-txns-asset-transfer-amount-isn't-zero";
        } else if (k == OutKind::NEW || k == OutKind::OWNER) {
            if (o.value != 0) return "bad-txns-asset-issued-amount-isn't-zero";
        } else if (k == OutKind::REISSUE) {
            if (f.enforce_values && block_check && o.value != 0) return "bad-txns-asset-reissued-amount-isn't-zero";
            if (mempool_check && o.value != 0) return "bad-mempool-txns-asset-reissued-amount-isn't-zero";
        }
    }
    if (add_tags && !burn_found(tx, p, Type::NULL_ADD_QUALIFIER, add_tags))
        return "bad-txns-tx-doesn't-contain-required-burn-fee-for-adding-tags";
    for (auto& [key, n] : tag_count) {
        const std::string& name = key.first;
        if (!name.empty() && name[0] == '$') {
            if (!transfer_names.count(name.substr(1) + "!"))
                return "bad-txns-tx-contains-restricted-asset-null-tx-without-asset-transfer";
        } else if (!transfer_names.count(name)) {
            return "bad-txns-tx-contains-qualifier-asset-null-tx-without-asset-transfer";
        }
    }
    for (auto& name : global_changes) {
        if (name.empty()) return "bad-txns-tx-contains-global-asset-null-tx-with-null-asset-name";
        if (!transfer_names.count(name.substr(1) + "!"))
            return "bad-txns-tx-contains-global-asset-null-tx-without-asset-transfer";
    }
    if (tx.is_coinbase()) {
        if (f.coinbase_assets)
            for (auto& o : tx.vout)
                if (asset_script_kind(o.script_pubkey) != OutKind::NONE || null_kind(o.script_pubkey) != NullKind::NONE)
                    return "bad-txns-coinbase-contains-asset-txes";
        return "";
    }
    bool new_restricted = false, restricted_reissue = false;
    const TxKind kind = tx_kind(tx);
    const Counts c = count_kinds(tx);
    AssetOut last;
    const bool last_ok = parse_asset_out(tx.vout.back().script_pubkey, last);
    switch (kind) {
        case TxKind::NEW: {
            if (!last_ok) return "bad-txns-issue-serialzation-failed";
            AssetOut owner;
            if (!parse_asset_out(tx.vout[tx.vout.size() - 2].script_pubkey, owner)) return "bad-txns-issue-owner-serialzation-failed";
            if (owner.name != last.name + "!") return "bad-txns-issue-owner-name-doesn't-match";
            const Type t = name_type(last.name);
            // two historical main-net issuances are accepted without their burn output (assets.h BAD_HASH)
            const std::string txid = tx.txid().hex();
            const bool grandfathered = txid == "e6cdd54445e6bf69710d54e4340a6486167f866575a878eaedecbb345da056ae" ||
                                       txid == "3ba63518dc12599f9b83449c8b5338e224caf363d0327f5156fa4b6efeca5724";
            if (!grandfathered && !burn_found(tx, p, t)) return "bad-txns-issue-burn-not-found";
            if (t == Type::SUB && !transfer_of(tx, parent_name(last.name) + "!"))
                return "bad-txns-issue-new-asset-missing-owner-asset";
            if (c.owners != 1 || c.issues != 1 || c.reissues > 0) return "bad-txns-failed-issue-asset-formatting-check";
            // IsNewOwnerTxValid
            if (std::memcmp(owner.h160, last.h160, 20) != 0) return "bad-txns-owner-address-mismatch";
            if (owner.name.size() < 1 + 3) return "bad-txns-owner-asset-length";
            const std::string err = check_new_asset(last);
            if (!err.empty()) return err;
            break;
        }
        case TxKind::REISSUE: {
            if (tx.vout.size() < 3) return "bad-txns-vout-size-to-small";
            if (!last_ok) return "bad-txns-reissue-serialization-failed";
            const Type t = name_type(last.name);
            const std::string root = t == Type::RESTRICTED ? last.name.substr(1) : last.name;
            if (!transfer_of(tx, root + "!")) return "bad-txns-reissue-owner-outpoint-not-found";
            if (!reissue_burn_found(tx, p)) return "bad-txns-reissue-burn-outpoint-not-found";
            if (c.owners > 0 || c.reissues != 1 || c.issues > 0) return "bad-txns-failed-reissue-asset-formatting-check";
            const std::string err = check_reissue(last, p.testnet);
            if (!err.empty()) return err;
            if (t == Type::RESTRICTED) {
                std::string v;
                if (tx_verifier(tx, v) < 0) return "bad-txns-reissue-restricted-verifier-Multiple verifier strings found in transaction";
                restricted_reissue = true;
            }
            break;
        }
        case TxKind::NEW_UNIQUE: {
            if (tx.vout.size() < 3) return "bad-txns-unique-vout-size-to-small";
            std::set<std::string> seen;
            std::string root;
            int n = 0;
            for (auto& o : tx.vout) {
                AssetOut a;
                if (new_out_type(o, &a) != Type::UNIQUE) continue;
                const std::string r = parent_name(a.name);
                if (root.empty()) root = r;
                if (r != root) return "bad-txns-issue-unique-asset-compare-failed";
                if (!seen.insert(a.name).second) return "bad-txns-issue-unique-duplicate-name-in-same-tx";
                ++n;
            }
            if (n == 0) return "bad-txns-issue-unique-asset-bad-outpoint-count";
            if (!burn_found(tx, p, Type::UNIQUE, n)) return "bad-txns-issue-unique-asset-burn-outpoints-not-found";
            if (!transfer_of(tx, root + "!")) return "bad-txns-issue-unique-asset-missing-owner-asset";
            if (c.owners > 0 || c.reissues > 0 || c.issues != n) return "bad-txns-failed-unique-asset-formatting-check";
            for (auto& o : tx.vout) {
                AssetOut a;
                if (new_out_type(o, &a) != Type::UNIQUE) continue;
                const std::string err = check_new_asset(a);
                if (!err.empty()) return "bad-txns-issue-unique" + err;
            }
            break;
        }
        case TxKind::NEW_MSGCHANNEL: {
            if (tx.vout.size() < 3) return "bad-txns-issue-msgchannel-vout-size-to-small";
            if (!burn_found(tx, p, Type::MSGCHANNEL)) return "bad-txns-issue-msgchannel-burn-not-found";
            if (!transfer_of(tx, parent_name(last.name) + "!")) return "bad-txns-issue-msg-channel-asset-bad-owner-asset";
            if (c.owners != 0 || c.issues != 1 || c.reissues > 0) return "bad-txns-failed-issue-msgchannel-asset-formatting-check";
            const std::string err = check_new_asset(last);
            if (!err.empty()) return "bad-txns-issue-msgchannel" + err;
            break;
        }
        case TxKind::NEW_QUALIFIER: {
            if (tx.vout.size() < 2) return "bad-txns-issue-qualifier-vout-size-to-small";
            const Type t = name_type(last.name);
            if (!burn_found(tx, p, t)) return "bad-txns-issue-qualifier-burn-not-found";
            if (t == Type::SUB_QUALIFIER && !transfer_of(tx, parent_name(last.name)))
                return "bad-txns-issue-sub-qualifier-parent-outpoint-not-found";
            if (c.owners != 0 || c.issues != 1 || c.reissues > 0) return "bad-txns-failed-issue-asset-formatting-check";
            const std::string err = check_new_asset(last);
            if (!err.empty()) return "bad-txns-issue-qualfier" + err;
            break;
        }
        case TxKind::NEW_RESTRICTED: {
            if (tx.vout.size() < 4) return "bad-txns-issue-restricted-vout-size-to-small";
            if (!burn_found(tx, p, Type::RESTRICTED)) return "bad-txns-issue-restricted-burn-not-found";
            if (!transfer_of(tx, parent_name(last.name).substr(1) + "!"))
                return "bad-txns-issue-restricted-root-owner-token-outpoint-not-found";
            std::string v;
            const int nv = tx_verifier(tx, v);
            if (nv < 0) return "Multiple verifier strings found in transaction";
            if (nv == 0) return "Verifier string not found";
            if (c.owners != 0 || c.issues != 1 || c.reissues > 0) return "bad-txns-failed-issue-asset-formatting-check";
            const std::string err = check_new_asset(last);
            if (!err.empty()) return "bad-txns-issue-restricted" + err;
            new_restricted = true;
            break;
        }
        case TxKind::NONE:
            for (auto& o : tx.vout) {
                const OutKind k = asset_script_kind(o.script_pubkey);
                if (k != OutKind::NONE) {
                    if (k != OutKind::TRANSFER) return "bad-txns-bad-asset-transaction";
                } else if (find_op(o.script_pubkey, kOpAsset) && o.script_pubkey[0] != kOpAsset) {
                    return "bad-txns-op-clore-asset-not-in-right-script-location";
                }
            }
            break;
    }
    if (has_verifier && !restricted_reissue && !new_restricted)
        return "bad-txns-tx-cointains-verifier-string-without-restricted-asset-issuance-or-reissuance";
    if (new_restricted && !has_verifier) return "bad-txns-tx-cointains-restricted-asset-issuance-without-verifier";
    return "";
}

// ------------------------------------------------------------------ state
namespace {

std::string key20(const u8 h[20]) { return std::string(reinterpret_cast<const char*>(h), 20); }

void write_meta(Writer& w, const Meta& m) {
    write_str(w, m.name);
    w.i64_(m.amount);
    w.u8_(u8(int8_t(m.units)));
    w.u8_(u8(int8_t(m.reissuable)));
    w.u8_(u8(int8_t(m.has_ipfs)));
    write_str(w, m.ipfs);
    w.i32_(m.height);
    w.u256(m.block);
}
Meta read_meta(Reader& r) {
    Meta m;
    m.name = read_str(r);
    m.amount = r.i64_();
    m.units = int8_t(r.u8_());
    m.reissuable = int8_t(r.u8_());
    m.has_ipfs = int8_t(r.u8_());
    m.ipfs = read_str(r);
    m.height = r.i32_();
    m.block = r.u256();
    return m;
}

}  // namespace

const Meta* State::find(const std::string& name) const {
    auto it = meta_.find(name);
    return it == meta_.end() ? nullptr : &it->second;
}

int64_t State::balance(const std::string& name, const u8 h160[20]) const {
    auto it = bal_.find({name, key20(h160)});
    return it == bal_.end() ? 0 : it->second;
}
bool State::has_tag(const std::string& q, const u8 h160[20]) const { return tags_.count({q, key20(h160)}) != 0; }
bool State::frozen(const std::string& r, const u8 h160[20]) const { return frozen_.count({r, key20(h160)}) != 0; }
const std::string* State::verifier(const std::string& r) const {
    auto it = verifier_.find(r);
    return it == verifier_.end() ? nullptr : &it->second;
}

void State::log(u8 kind, const std::string& a, const std::string& b) {
    Op op;
    op.kind = kind;
    op.a = a;
    op.b = b;
    Writer w;
    switch (kind) {
        case 0: {
            auto it = meta_.find(a);
            op.had = it != meta_.end();
            if (op.had) write_meta(w, it->second);
            break;
        }
        case 1: {
            auto it = bal_.find({a, b});
            op.had = it != bal_.end();
            if (op.had) w.i64_(it->second);
            break;
        }
        case 2: op.had = tags_.count({a, b}) != 0; break;
        case 3: op.had = frozen_.count({a, b}) != 0; break;
        case 4: op.had = global_.count(a) != 0; break;
        case 5: {
            auto it = verifier_.find(a);
            op.had = it != verifier_.end();
            if (op.had) write_str(w, it->second);
            break;
        }
    }
    op.old = std::move(w.buf);
    dirty_.insert({kind, {a, b}});
    journal_.push_back(std::move(op));
}

void State::for_each_dirty(
    const std::function<void(u8, const std::string&, const std::string&, const Bytes*)>& f) const {
    for (auto& [kind, k] : dirty_) {
        Writer w;
        bool has = false;
        switch (kind) {
            case 0: {
                auto it = meta_.find(k.first);
                if ((has = it != meta_.end())) write_meta(w, it->second);
                break;
            }
            case 1: {
                auto it = bal_.find(k);
                if ((has = it != bal_.end())) w.i64_(it->second);
                break;
            }
            case 2: has = tags_.count(k) != 0; break;
            case 3: has = frozen_.count(k) != 0; break;
            case 4: has = global_.count(k.first) != 0; break;
            case 5: {
                auto it = verifier_.find(k.first);
                if ((has = it != verifier_.end())) write_str(w, it->second);
                break;
            }
        }
        f(kind, k.first, k.second, has ? &w.buf : nullptr);
    }
}

void State::mark_all_dirty() {
    for (auto& kv : meta_) dirty_.insert({0, {kv.first, ""}});
    for (auto& kv : bal_) dirty_.insert({1, kv.first});
    for (auto& k : tags_) dirty_.insert({2, k});
    for (auto& k : frozen_) dirty_.insert({3, k});
    for (auto& k : global_) dirty_.insert({4, {k, ""}});
    for (auto& kv : verifier_) dirty_.insert({5, {kv.first, ""}});
}

bool State::load_entry(u8 kind, const std::string& a, const std::string& b, const Bytes& value) {
    try {
        Reader r(value);
        switch (kind) {
            case 0: meta_[a] = read_meta(r); break;
            case 1: bal_[{a, b}] = r.i64_(); break;
            case 2: tags_.insert({a, b}); break;
            case 3: frozen_.insert({a, b}); break;
            case 4: global_.insert(a); break;
            case 5: verifier_[a] = read_str(r); break;
            default: return false;
        }
    } catch (const std::exception&) {
        return false;
    }
    return true;
}

void State::set_meta(const Meta& m) {
    log(0, m.name, "");
    meta_[m.name] = m;
}
void State::erase_meta(const std::string& name) {
    log(0, name, "");
    meta_.erase(name);
}
void State::add_balance(const std::string& name, const u8 h160[20], int64_t delta) {
    const std::string k = key20(h160);
    log(1, name, k);
    int64_t& v = bal_[{name, k}];
    v += delta;
    if (v == 0) bal_.erase({name, k});
}
void State::set_tag(const std::string& q, const u8 h160[20], bool on) {
    log(2, q, key20(h160));
    if (on) tags_.insert({q, key20(h160)});
    else tags_.erase({q, key20(h160)});
}
void State::set_frozen(const std::string& r, const u8 h160[20], bool on) {
    log(3, r, key20(h160));
    if (on) frozen_.insert({r, key20(h160)});
    else frozen_.erase({r, key20(h160)});
}
void State::set_global(const std::string& r, bool on) {
    log(4, r, "");
    if (on) global_.insert(r);
    else global_.erase(r);
}
void State::set_verifier(const std::string& r, const std::string& v) {
    log(5, r, "");
    verifier_[r] = v;
}

void State::restore(const Op& op) {
    dirty_.insert({op.kind, {op.a, op.b}});
    Reader r(op.old);
    switch (op.kind) {
        case 0:
            if (op.had) meta_[op.a] = read_meta(r);
            else meta_.erase(op.a);
            break;
        case 1:
            if (op.had) bal_[{op.a, op.b}] = r.i64_();
            else bal_.erase({op.a, op.b});
            break;
        case 2:
            if (op.had) tags_.insert({op.a, op.b});
            else tags_.erase({op.a, op.b});
            break;
        case 3:
            if (op.had) frozen_.insert({op.a, op.b});
            else frozen_.erase({op.a, op.b});
            break;
        case 4:
            if (op.had) global_.insert(op.a);
            else global_.erase(op.a);
            break;
        case 5:
            if (op.had) verifier_[op.a] = read_str(r);
            else verifier_.erase(op.a);
            break;
    }
}

Bytes State::journal_since(size_t m) const {
    Writer w;
    w.compact_size(journal_.size() - m);
    for (size_t i = m; i < journal_.size(); ++i) {
        const Op& op = journal_[i];
        w.u8_(op.kind);
        write_str(w, op.a);
        write_str(w, op.b);
        w.u8_(op.had ? 1 : 0);
        w.var_bytes(op.old);
    }
    return w.buf;
}

void State::rollback_to(size_t m) {
    while (journal_.size() > m) {
        restore(journal_.back());
        journal_.pop_back();
    }
}

bool State::undo(const Bytes& record) {
    std::vector<Op> ops;
    try {
        Reader r(record);
        const u64 n = r.compact_size();
        ops.resize(size_t(n));
        for (auto& op : ops) {
            op.kind = r.u8_();
            op.a = read_str(r);
            op.b = read_str(r);
            op.had = r.u8_() != 0;
            op.old = r.var_bytes();
            if (op.kind > 5) return false;
        }
    } catch (const std::exception&) {
        return false;
    }
    for (auto it = ops.rbegin(); it != ops.rend(); ++it) restore(*it);
    return true;
}

Bytes State::serialize() const {
    Writer w;
    w.u256(best_block);
    w.compact_size(meta_.size());
    for (auto& [k, m] : meta_) write_meta(w, m);
    w.compact_size(bal_.size());
    for (auto& [k, v] : bal_) {
        write_str(w, k.first);
        write_str(w, k.second);
        w.i64_(v);
    }
    for (const std::set<AddrKey>* s : {&tags_, &frozen_}) {
        w.compact_size(s->size());
        for (auto& k : *s) {
            write_str(w, k.first);
            write_str(w, k.second);
        }
    }
    w.compact_size(global_.size());
    for (auto& g : global_) write_str(w, g);
    w.compact_size(verifier_.size());
    for (auto& [k, v] : verifier_) {
        write_str(w, k);
        write_str(w, v);
    }
    return w.buf;
}

bool State::deserialize(const Bytes& b) {
    State s;
    try {
        Reader r(b);
        s.best_block = r.u256();
        for (u64 n = r.compact_size(); n--;) {
            Meta m = read_meta(r);
            s.meta_[m.name] = m;
        }
        for (u64 n = r.compact_size(); n--;) {
            std::string a = read_str(r), k = read_str(r);
            s.bal_[{a, k}] = r.i64_();
        }
        for (std::set<AddrKey>* set : {&s.tags_, &s.frozen_})
            for (u64 n = r.compact_size(); n--;) {
                std::string a = read_str(r), k = read_str(r);
                set->insert({a, k});
            }
        for (u64 n = r.compact_size(); n--;) s.global_.insert(read_str(r));
        for (u64 n = r.compact_size(); n--;) {
            std::string a = read_str(r);
            s.verifier_[a] = read_str(r);
        }
        if (!r.empty()) return false;
    } catch (const std::exception&) {
        return false;
    }
    *this = std::move(s);
    return true;
}

// ------------------------------------------------------------------ contextual checks
namespace {

bool encoded_ok(const std::string& raw, bool msg_active) {
    const std::string e = encode_asset_data(raw);
    if (e.size() == 46 && e.compare(0, 2, "Qm") == 0) return true;
    return msg_active && raw.size() == 32;
}

// ContextualCheckVerifierString with an optional address (empty = syntax + qualifiers exist)
std::string check_verifier_ctx(const State& st, const std::string& verifier, const u8* h160) {
    if (verifier == "true") return "";
    std::set<std::string> found;
    std::string err;
    if (!check_verifier(verifier, found, err)) return err;
    for (auto& q : found)
        if (!st.exists("#" + q)) return "bad-txns-null-verifier-contains-non-issued-qualifier";
    if (!h160) return "";
    std::map<std::string, bool> vals;
    for (auto& q : found) vals[q] = st.has_tag("#" + q, h160);
    try {
        if (!bool_expr(verifier, vals)) return "bad-txns-null-verifier-address-failed-verification";
    } catch (const std::runtime_error&) {
        return "bad-txns-null-verifier-failed-contexual-syntax-check";
    }
    return "";
}

std::string check_new_ctx(const State& st, const AssetOut& a, const Flags& f, const std::set<std::string>* pending) {
    if (!f.assets) return "bad-txns-new-asset-when-assets-is-not-active";
    std::string err = check_new_asset(a);
    if (!err.empty()) return err;
    if (st.exists(a.name)) return "Invalid parameter: asset_name '" + a.name + "' has already been used";
    if (pending && pending->count(a.name)) return "Asset with this name is already in the mempool";
    if (a.has_ipfs && a.ipfs.size() != 34) {
        if (!f.msg_restricted || a.ipfs.size() != 32)
            return "Invalid parameter: ipfs_hash must be 46 characters. Txid must be valid 64 character hash";
    }
    if (a.has_ipfs && !encoded_ok(a.ipfs, f.msg_restricted))
        return "Invalid parameter: ipfs_hash is not valid, or txid hash is not the right length";
    return "";
}

}  // namespace

std::string check_tx_contextual(const Transaction& tx, const std::vector<const Coin*>& spent, const State& st,
                                const Flags& f, const std::set<std::string>* pending_names) {
    std::map<std::string, int64_t> in_total, out_total;
    for (size_t i = 0; i < spent.size(); ++i) {
        const Bytes& spk = spent[i]->out.script_pubkey;
        if (asset_script_kind(spk) == OutKind::NONE) continue;
        AssetOut a;
        if (!parse_asset_out(spk, a)) return "bad-txns-failed-to-get-asset-from-script";
        in_total[a.name] += a.amount;
        if (name_type(a.name) == Type::RESTRICTED && st.frozen(a.name, a.h160))
            return "bad-txns-restricted-asset-transfer-from-frozen-address";
    }
    for (auto& o : tx.vout) {
        const Bytes& spk = o.script_pubkey;
        const OutKind k = asset_script_kind(spk);
        if (k != OutKind::NONE && !f.assets) return "bad-txns-is-asset-and-asset-not-active";
        const NullKind nk = null_kind(spk);
        if (nk != NullKind::NONE) {
            if (!f.msg_restricted) return "bad-tx-null-asset-data-before-restricted-assets-activated";
            if (nk == NullKind::TAG) {
                std::string name;
                int flag;
                u8 h[20];
                if (!parse_null_tag(spk, name, flag, h)) return "bad-txns-null-asset-data-serialization";
                const Type t = name_type(name);
                if (t == Type::QUALIFIER || t == Type::SUB_QUALIFIER) {
                    const bool has = st.has_tag(name, h);
                    if (flag == 1 && has) return "bad-txns-null-data-add-qualifier-when-already-assigned";
                    if (flag == 0 && !has) return "bad-txns-null-data-removing-qualifier-when-not-assigned";
                } else if (t == Type::RESTRICTED) {
                    const bool frz = st.frozen(name, h);
                    if (flag == 1 && frz) return "bad-txns-null-data-freeze-address-when-already-frozen";
                    if (flag == 0 && !frz) return "bad-txns-null-data-unfreeze-address-when-not-frozen";
                } else {
                    return "bad-txns-null-asset-data-on-non-restricted-or-qualifier-asset";
                }
            } else if (nk == NullKind::GLOBAL) {
                std::string name;
                int flag;
                if (!parse_null_global(spk, name, flag)) return "bad-txns-null-global-asset-data-serialization";
                const bool g = st.global_frozen(name);
                if (flag == 1 && g) return "bad-txns-null-data-global-freeze-when-already-frozen";
                if (flag == 0 && !g) return "bad-txns-null-data-global-unfreeze-when-not-frozen";
            } else {
                std::string v;
                if (!parse_null_verifier(spk, v)) return "bad-txns-null-verifier-data-serialization";
                const std::string err = check_verifier_ctx(st, v, nullptr);
                if (!err.empty()) return err;
            }
        }
        if (k == OutKind::TRANSFER) {
            AssetOut a;
            if (!parse_asset_out(spk, a)) return "bad-tx-asset-transfer-bad-deserialize";
            const Type t = name_type(a.name);
            if (t == Type::INVALID) return "Invalid parameter: asset_name must only consist of valid characters";
            if (a.amount <= 0) return "Invalid parameter: asset amount can't be equal to or less than zero.";
            if (f.msg_restricted) {
                if (a.message.empty() && a.expire > 0)
                    return "Invalid parameter: asset transfer expiration time requires a message to be attached to the transfer";
                if (a.expire < 0) return "Invalid parameter: expiration time must be a positive value";
                if (!a.message.empty() && !encoded_ok(a.message, true))
                    return "Invalid parameter: ipfs_hash is not valid, or txid hash is not the right length";
            }
            if (t == Type::MSGCHANNEL && !f.msg_restricted) return "bad-txns-transfer-msgchannel-before-messaging-is-active";
            if (t == Type::RESTRICTED) {
                if (!f.msg_restricted) return "bad-txns-transfer-restricted-before-it-is-active";
                if (st.global_frozen(a.name)) return "bad-txns-transfer-restricted-asset-that-is-globally-restricted";
                const std::string* v = st.verifier(a.name);
                if (!v) return "Verifier String doesn't exist for asset: " + a.name;
                const std::string err = check_verifier_ctx(st, *v, a.h160);
                if (!err.empty()) return err;
            }
            if ((t == Type::QUALIFIER || t == Type::SUB_QUALIFIER) && !f.msg_restricted)
                return "bad-txns-transfer-qualifier-before-it-is-active";
            out_total[a.name] += a.amount;
            if (t == Type::OWNER) {
                if (a.amount != kOwnerAmount) return "bad-txns-transfer-owner-amount-was-not-1";
            } else {
                const Meta* m = st.find(a.name);
                if (!m) return "bad-txns-transfer-asset-not-exist";
                if (!amount_fits_units(a.amount, m->units)) return "bad-txns-transfer-asset-amount-not-match-units";
            }
        }
    }
    const TxKind kind = tx_kind(tx);
    AssetOut last;
    const bool last_ok = parse_asset_out(tx.vout.back().script_pubkey, last);
    switch (kind) {
        case TxKind::NEW: {
            if (!last_ok) return "bad-txns-issue-serialzation-failed";
            const std::string err = check_new_ctx(st, last, f, pending_names);
            if (!err.empty()) return err;
            break;
        }
        case TxKind::REISSUE: {
            if (!last_ok) return "bad-txns-reissue-serialzation-failed";
            std::string err = check_reissue(last, false);
            const Meta* prev = st.find(last.name);
            if (err.empty() && !prev) err = "Unable to reissue asset: asset_name '" + last.name + "' doesn't exist in the database";
            if (err.empty() && !prev->reissuable) err = "Unable to reissue asset: reissuable is set to false";
            if (err.empty() && prev->amount + last.amount > kMaxMoneyAssets)
                err = "Unable to reissue asset: asset_name '" + last.name + "' the amount trying to reissue is to large";
            if (err.empty() && !amount_fits_units(last.amount, prev->units))
                err = "Unable to reissue asset: amount must be divisible by the smaller unit assigned to the asset";
            if (err.empty() && last.units < prev->units && last.units != -1)
                err = "Unable to reissue asset: unit must be larger than current unit selection";
            if (err.empty() && !last.ipfs.empty() && last.ipfs.size() != 34 && f.msg_restricted && last.ipfs.size() != 32)
                err = "Invalid parameter: ipfs_hash must be 34 bytes, Txid must be 32 bytes";
            if (err.empty() && !last.ipfs.empty() && !encoded_ok(last.ipfs, f.msg_restricted))
                err = "Invalid parameter: ipfs_hash is not valid, or txid hash is not the right length";
            if (err.empty() && name_type(last.name) == Type::RESTRICTED && last.amount > 0) {
                std::string v;
                const int nv = tx_verifier(tx, v);
                if (nv < 0) return "bad-txns-reissue-contextual-Multiple verifier strings found in transaction";
                const std::string* cur = nv ? &v : st.verifier(last.name);
                if (!cur) err = "failed to get verifier string from a restricted asset, database is out of sync";
                else err = check_verifier_ctx(st, *cur, last.h160);
            }
            if (!err.empty()) return "bad-txns-reissue-contextual-" + err;
            break;
        }
        case TxKind::NEW_UNIQUE:
            for (auto& o : tx.vout) {
                AssetOut a;
                if (new_out_type(o, &a) != Type::UNIQUE) continue;
                const std::string err = check_new_ctx(st, a, f, pending_names);
                if (!err.empty()) return "bad-txns-issue-unique-contextual-" + err;
            }
            break;
        case TxKind::NEW_MSGCHANNEL: {
            if (!f.msg_restricted) return "bad-txns-issue-msgchannel-before-messaging-is-active";
            const std::string err = check_new_ctx(st, last, f, pending_names);
            if (!err.empty()) return "bad-txns-issue-msgchannel-contextual-" + err;
            break;
        }
        case TxKind::NEW_QUALIFIER: {
            if (!f.msg_restricted) return "bad-txns-issue-qualifier-before-it-is-active";
            const std::string err = check_new_ctx(st, last, f, pending_names);
            if (!err.empty()) return "bad-txns-issue-qualfier-contextual" + err;
            break;
        }
        case TxKind::NEW_RESTRICTED: {
            if (!f.msg_restricted) return "bad-txns-issue-restricted-before-it-is-active";
            std::string err = check_new_ctx(st, last, f, pending_names);
            if (!err.empty()) return "bad-txns-issue-restricted-contextual" + err;
            std::string v;
            if (tx_verifier(tx, v) != 1) return "bad-txns-issue-restricted-verifier-search-Verifier string not found";
            err = check_verifier_ctx(st, v, last.h160);
            if (!err.empty()) return err;
            break;
        }
        case TxKind::NONE:
            for (auto& o : tx.vout) {
                const OutKind k = asset_script_kind(o.script_pubkey);
                if (k != OutKind::NONE) {
                    if (k != OutKind::TRANSFER) return "bad-txns-bad-asset-transaction";
                } else if (find_op(o.script_pubkey, kOpAsset)) {
                    if (!f.msg_restricted) return "bad-txns-bad-asset-script";
                    if (o.script_pubkey[0] != kOpAsset) return "bad-txns-op-clore-asset-not-in-right-script-location";
                }
            }
            break;
    }
    for (auto& [name, amount] : out_total) {
        auto it = in_total.find(name);
        if (it == in_total.end())
            return "bad-tx-inputs-outputs-mismatch Bad Transaction - Trying to create outpoint for asset that you don't have: " + name;
        if (it->second != amount) return "bad-tx-inputs-outputs-mismatch Bad Transaction - Assets would be burnt " + name;
    }
    if (out_total.size() != in_total.size()) return "bad-tx-asset-inputs-size-does-not-match-outputs-size";
    return "";
}

void apply_tx(const Transaction& tx, const std::vector<Coin>& spent, int height, const Uint256& block_hash,
              State& st) {
    // SpendCoin: the spent asset outputs leave their addresses
    for (auto& c : spent) {
        AssetOut a;
        if (asset_script_kind(c.out.script_pubkey) != OutKind::NONE && parse_asset_out(c.out.script_pubkey, a))
            st.add_balance(a.name, a.h160, -a.amount);
    }
    auto new_meta = [&](const AssetOut& a) {
        Meta m;
        m.name = a.name;
        m.amount = a.amount;
        m.units = a.units;
        m.reissuable = a.reissuable;
        m.has_ipfs = a.has_ipfs;
        m.ipfs = a.ipfs;
        m.height = height;
        m.block = block_hash;
        st.set_meta(m);
    };
    const TxKind kind = tx_kind(tx);
    std::string verifier;
    const bool has_verifier = tx_verifier(tx, verifier) == 1;
    for (auto& o : tx.vout) {
        const Bytes& spk = o.script_pubkey;
        AssetOut a;
        const OutKind k = asset_script_kind(spk);
        if (k != OutKind::NONE && parse_asset_out(spk, a)) {
            switch (k) {
                case OutKind::NEW:
                    if (kind != TxKind::NONE && kind != TxKind::REISSUE) new_meta(a);
                    st.add_balance(a.name, a.h160, a.amount);
                    if (kind == TxKind::NEW_RESTRICTED && has_verifier) st.set_verifier(a.name, verifier);
                    break;
                case OutKind::OWNER: {
                    if (kind == TxKind::NEW) {
                        AssetOut owner = a;
                        owner.units = 0;
                        owner.reissuable = 0;
                        owner.has_ipfs = 0;
                        owner.ipfs.clear();
                        new_meta(owner);
                    }
                    st.add_balance(a.name, a.h160, kOwnerAmount);
                    break;
                }
                case OutKind::TRANSFER:
                    if (a.amount > 0) st.add_balance(a.name, a.h160, a.amount);
                    break;
                case OutKind::REISSUE:
                    if (kind == TxKind::REISSUE) {
                        if (const Meta* prev = st.find(a.name)) {
                            Meta m = *prev;
                            m.amount += a.amount;
                            m.reissuable = a.reissuable;
                            if (a.units != -1) m.units = a.units;
                            if (!a.ipfs.empty()) {
                                m.has_ipfs = 1;
                                m.ipfs = a.ipfs;
                            }
                            st.set_meta(m);
                            if (name_type(a.name) == Type::RESTRICTED && has_verifier) st.set_verifier(a.name, verifier);
                        }
                    }
                    st.add_balance(a.name, a.h160, a.amount);
                    break;
                default: break;
            }
        }
        switch (null_kind(spk)) {
            case NullKind::TAG: {
                std::string name;
                int flag;
                u8 h[20];
                if (!parse_null_tag(spk, name, flag, h)) break;
                const Type t = name_type(name);
                if (t == Type::RESTRICTED) st.set_frozen(name, h, flag != 0);
                else if (t == Type::QUALIFIER || t == Type::SUB_QUALIFIER) st.set_tag(name, h, flag != 0);
                break;
            }
            case NullKind::GLOBAL: {
                std::string name;
                int flag;
                if (parse_null_global(spk, name, flag)) st.set_global(name, flag != 0);
                break;
            }
            default: break;
        }
    }
}

// ------------------------------------------------------------------ display forms
std::string encode_asset_data(const std::string& raw) {
    if (raw.size() == 34) return base58_encode(Bytes(raw.begin(), raw.end()));
    if (raw.size() == 32) {
        static const char* hex = "0123456789abcdef";
        std::string s;
        for (unsigned char c : raw) {
            s += hex[c >> 4];
            s += hex[c & 15];
        }
        return s;
    }
    return "";
}

std::string decode_asset_data(const std::string& s) {
    if (s.size() == 46) {
        Bytes b;
        if (!base58_decode(s, b)) return "";
        return std::string(b.begin(), b.end());
    }
    if (s.size() == 64) {
        std::string out;
        for (size_t i = 0; i < 64; i += 2) {
            auto nib = [](char c) -> int {
                if (c >= '0' && c <= '9') return c - '0';
                if (c >= 'a' && c <= 'f') return c - 'a' + 10;
                if (c >= 'A' && c <= 'F') return c - 'A' + 10;
                return -1;
            };
            const int hi = nib(s[i]), lo = nib(s[i + 1]);
            if (hi < 0 || lo < 0) return "";
            out += char(hi * 16 + lo);
        }
        return out;
    }
    return "";
}

}  // namespace nodexa::assets
