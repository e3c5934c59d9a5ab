#include "script.hpp"

#include <utility>

#include "../crypto/sha256.hpp"

namespace nodexa {

ScriptBuilder& ScriptBuilder::push_data(const Bytes& d) {
    if (d.size() < OP_PUSHDATA1) {
        s.push_back(u8(d.size()));
    } else if (d.size() <= 0xff) {
        s.push_back(OP_PUSHDATA1);
        s.push_back(u8(d.size()));
    } else if (d.size() <= 0xffff) {
        s.push_back(OP_PUSHDATA2);
        s.push_back(u8(d.size()));
        s.push_back(u8(d.size() >> 8));
    } else {
        s.push_back(OP_PUSHDATA4);
        u8 b[4];
        store_le32(b, u32(d.size()));
        s.insert(s.end(), b, b + 4);
    }
    s.insert(s.end(), d.begin(), d.end());
    return *this;
}

Bytes ScriptBuilder::scriptnum(int64_t value) {
    Bytes result;
    if (value == 0) return result;
    const bool neg = value < 0;
    u64 absvalue = neg ? u64(-value) : u64(value);
    while (absvalue) {
        result.push_back(u8(absvalue & 0xff));
        absvalue >>= 8;
    }
    if (result.back() & 0x80) result.push_back(neg ? 0x80 : 0);
    else if (neg) result.back() |= 0x80;
    return result;
}

ScriptBuilder& ScriptBuilder::push_int(int64_t v) {
    if (v == -1 || (v >= 1 && v <= 16)) s.push_back(u8(v + (OP_1 - 1)));
    else if (v == 0) s.push_back(OP_0);
    else push_data(scriptnum(v));
    return *this;
}

ScriptBuilder& ScriptBuilder::push_num(int64_t v) { return push_data(scriptnum(v)); }

// ---------------- Base58 ----------------
static const char* kB58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";

std::string base58_encode(const Bytes& in) {
    size_t zeros = 0;
    while (zeros < in.size() && in[zeros] == 0) ++zeros;
    std::vector<u8> b58((in.size() - zeros) * 138 / 100 + 1, 0);
    size_t length = 0;
    for (size_t i = zeros; i < in.size(); ++i) {
        int carry = in[i];
        size_t j = 0;
        for (auto it = b58.rbegin(); (carry != 0 || j < length) && it != b58.rend(); ++it, ++j) {
            carry += 256 * (*it);
            *it = u8(carry % 58);
            carry /= 58;
        }
        length = j;
    }
    auto it = b58.begin() + (b58.size() - length);
    while (it != b58.end() && *it == 0) ++it;
    std::string out(zeros, '1');
    for (; it != b58.end(); ++it) out += kB58[*it];
    return out;
}

bool base58_decode(const std::string& s, Bytes& out) {
    size_t i = 0, zeros = 0;
    while (i < s.size() && s[i] == '1') { ++zeros; ++i; }
    std::vector<u8> b256((s.size() - i) * 733 / 1000 + 1, 0);
    size_t length = 0;
    for (; i < s.size(); ++i) {
        const char* p = std::strchr(kB58, s[i]);
        if (!p || !*p) return false;
        int carry = int(p - kB58);
        size_t j = 0;
        for (auto it = b256.rbegin(); (carry != 0 || j < length) && it != b256.rend(); ++it, ++j) {
            carry += 58 * (*it);
            *it = u8(carry % 256);
            carry /= 256;
        }
        length = j;
    }
    auto it = b256.begin() + (b256.size() - length);
    out.assign(zeros, 0);
    out.insert(out.end(), it, b256.end());
    return true;
}

std::string base58check_encode(const Bytes& payload) {
    Bytes d = payload;
    u8 h[32];
    sha256d(d.data(), d.size(), h);
    d.insert(d.end(), h, h + 4);
    return base58_encode(d);
}

bool base58check_decode(const std::string& s, Bytes& payload) {
    Bytes d;
    if (!base58_decode(s, d) || d.size() < 4) return false;
    u8 h[32];
    sha256d(d.data(), d.size() - 4, h);
    if (std::memcmp(h, d.data() + d.size() - 4, 4) != 0) return false;
    payload.assign(d.begin(), d.end() - 4);
    return true;
}

bool address_to_script(const std::string& addr, u8 pkh, u8 sh, Bytes& script) {
    Bytes p;
    if (!base58check_decode(addr, p) || p.size() != 21) return false;
    if (p[0] == pkh) {
        script = {OP_DUP, OP_HASH160, 20};
        script.insert(script.end(), p.begin() + 1, p.end());
        script.push_back(OP_EQUALVERIFY);
        script.push_back(OP_CHECKSIG);
        return true;
    }
    if (p[0] == sh) {
        script = {OP_HASH160, 20};
        script.insert(script.end(), p.begin() + 1, p.end());
        script.push_back(OP_EQUAL);
        return true;
    }
    return false;
}

std::string script_to_address(const Bytes& s, u8 pkh, u8 sh) {
    if (s.size() == 25 && s[0] == OP_DUP && s[1] == OP_HASH160 && s[2] == 20 && s[23] == OP_EQUALVERIFY &&
        s[24] == OP_CHECKSIG) {
        Bytes p{pkh};
        p.insert(p.end(), s.begin() + 3, s.begin() + 23);
        return base58check_encode(p);
    }
    if (s.size() == 23 && s[0] == OP_HASH160 && s[1] == 20 && s[22] == OP_EQUAL) {
        Bytes p{sh};
        p.insert(p.end(), s.begin() + 2, s.begin() + 22);
        return base58check_encode(p);
    }
    return "";
}

// ---------------- RIPEMD-160 (Dobbertin, Bosselaers, Preneel 1996) ----------------
namespace {
constexpr inline u32 rf(int j, u32 x, u32 y, u32 z) {
    switch (j / 16) {
        case 0: return x ^ y ^ z;
        case 1: return (x & y) | (~x & z);
        case 2: return (x | ~y) ^ z;
        case 3: return (x & z) | (y & ~z);
        default: return x ^ (y | ~z);
    }
}
constexpr u32 KL[5] = {0x00000000, 0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xA953FD4E};
constexpr u32 KR[5] = {0x50A28BE6, 0x5C4DD124, 0x6D703EF3, 0x7A6D76E9, 0x00000000};
constexpr int RL[80] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 7, 4, 13, 1, 10, 6, 15, 3, 12, 0, 9,
                    5, 2, 14, 11, 8, 3, 10, 14, 4, 9, 15, 8, 1, 2, 7, 0, 6, 13, 11, 5, 12, 1, 9, 11, 10, 0, 8,
                    12, 4, 13, 3, 7, 15, 14, 5, 6, 2, 4, 0, 5, 9, 7, 12, 2, 10, 14, 1, 3, 8, 11, 6, 15, 13};
constexpr int RR[80] = {5, 14, 7, 0, 9, 2, 11, 4, 13, 6, 15, 8, 1, 10, 3, 12, 6, 11, 3, 7, 0, 13, 5, 10, 14, 15, 8,
                    12, 4, 9, 1, 2, 15, 5, 1, 3, 7, 14, 6, 9, 11, 8, 12, 2, 10, 0, 4, 13, 8, 6, 4, 1, 3, 11,
                    15, 0, 5, 12, 2, 13, 9, 7, 10, 14, 12, 15, 10, 4, 1, 5, 8, 7, 6, 2, 13, 14, 0, 3, 9, 11};
constexpr int SL[80] = {11, 14, 15, 12, 5, 8, 7, 9, 11, 13, 14, 15, 6, 7, 9, 8, 7, 6, 8, 13, 11, 9, 7, 15, 7, 12, 15,
                    9, 11, 7, 13, 12, 11, 13, 6, 7, 14, 9, 13, 15, 14, 8, 13, 6, 5, 12, 7, 5, 11, 12, 14, 15,
                    14, 15, 9, 8, 9, 14, 5, 6, 8, 6, 5, 12, 9, 15, 5, 11, 6, 8, 13, 12, 5, 12, 13, 14, 11, 8,
                    5, 6};
constexpr int SR[80] = {8, 9, 9, 11, 13, 15, 15, 5, 7, 7, 8, 11, 14, 14, 12, 6, 9, 13, 15, 7, 12, 8, 9, 11, 7, 7, 12,
                    7, 6, 15, 13, 11, 9, 7, 15, 11, 8, 6, 6, 14, 12, 13, 5, 14, 13, 13, 7, 5, 15, 5, 8, 11, 14,
                    14, 6, 14, 6, 9, 12, 9, 12, 5, 15, 8, 8, 5, 12, 9, 12, 5, 14, 6, 8, 13, 6, 5, 15, 13, 11,
                    11};

// Both lines fully unrolled at compile time (the step index J is a template argument,
// so the boolean function, message word and rotation fold to constants).
template <int J>
inline void rmd_step(u32 (&l)[5], u32 (&r)[5], const u32 (&X)[16]) {
    u32 t = rotl32(l[0] + rf(J, l[1], l[2], l[3]) + X[RL[J]] + KL[J / 16], SL[J]) + l[4];
    l[0] = l[4]; l[4] = l[3]; l[3] = rotl32(l[2], 10); l[2] = l[1]; l[1] = t;
    t = rotl32(r[0] + rf(79 - J, r[1], r[2], r[3]) + X[RR[J]] + KR[J / 16], SR[J]) + r[4];
    r[0] = r[4]; r[4] = r[3]; r[3] = rotl32(r[2], 10); r[2] = r[1]; r[1] = t;
}

template <int... J>
inline void rmd_steps(std::integer_sequence<int, J...>, u32 (&l)[5], u32 (&r)[5], const u32 (&X)[16]) {
    (rmd_step<J>(l, r, X), ...);
}

void rmd_compress(u32 h[5], const u8* block) {
    u32 X[16];
    for (int i = 0; i < 16; ++i) X[i] = load_le32(block + 4 * i);
    u32 l[5] = {h[0], h[1], h[2], h[3], h[4]};
    u32 r[5] = {h[0], h[1], h[2], h[3], h[4]};
    rmd_steps(std::make_integer_sequence<int, 80>{}, l, r, X);
    const u32 t = h[1] + l[2] + r[3];
    h[1] = h[2] + l[3] + r[4];
    h[2] = h[3] + l[4] + r[0];
    h[3] = h[4] + l[0] + r[1];
    h[4] = h[0] + l[1] + r[2];
    h[0] = t;
}
}  // namespace

void ripemd160(const u8* data, size_t n, u8 out[20]) {
    u32 h[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
    size_t i = 0;
    for (; i + 64 <= n; i += 64) rmd_compress(h, data + i);
    u8 tail[128] = {0};
    const size_t rem = n - i;
    if (rem) std::memcpy(tail, data + i, rem);
    tail[rem] = 0x80;
    const size_t tl = (rem < 56) ? 64 : 128;
    store_le64(tail + tl - 8, u64(n) * 8);
    rmd_compress(h, tail);
    if (tl == 128) rmd_compress(h, tail + 64);
    for (int k = 0; k < 5; ++k) store_le32(out + 4 * k, h[k]);
}

void hash160(const u8* data, size_t n, u8 out[20]) {
    u8 s[32];
    sha256(data, n, s);
    ripemd160(s, 32, out);
}

}  // namespace nodexa
