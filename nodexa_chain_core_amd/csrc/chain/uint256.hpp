// 256-bit blob (uint256) and 256-bit unsigned arithmetic (arith_uint256).
//
// Parity: uint256 / GetHex / SetHex / GetNibble (src/uint256.h:125-136,
// src/uint256.cpp:24-27); arith_uint256 incl. SetCompact / GetCompact
// (src/arith_uint256.cpp:209-260). Arithmetic is modulo 2^256 exactly like the
// reference's base_uint (DarkGravityWave relies on that wrap-around for the
// regtest 0x7fff.. limit, src/pow.cpp:57,90-91).
#pragma once

#include <algorithm>

#include "../crypto/keccak.hpp"
#include "../util/common.hpp"

namespace nodexa {

struct Uint256 {
    u8 data[32];
    Uint256() { std::memset(data, 0, 32); }
    static Uint256 from_bytes(const u8* p) { Uint256 r; std::memcpy(r.data, p, 32); return r; }
    bool is_null() const { for (u8 b : data) if (b) return false; return true; }
    void set_null() { std::memset(data, 0, 32); }
    bool operator==(const Uint256& o) const { return std::memcmp(data, o.data, 32) == 0; }
    bool operator!=(const Uint256& o) const { return !(*this == o); }
    bool operator<(const Uint256& o) const { return std::memcmp(data, o.data, 32) < 0; }
    std::string hex() const;                      // GetHex: reversed byte order
    static Uint256 from_hex(const std::string&);  // uint256S: accepts 0x, short strings
    int nibble(int index) const {                 // GetNibble (src/uint256.h:130-136)
        index = 63 - index;
        return (index % 2 == 1) ? (data[index / 2] >> 4) : (data[index / 2] & 0x0F);
    }
    u64 cheap_hash() const { return load_le64(data); }
    // ethash <-> node byte order (to_hash256(GetHex()) / uint256S(to_hex())).
    Hash256 to_progpow() const { Hash256 h; for (int i = 0; i < 32; ++i) h.bytes[i] = data[31 - i]; return h; }
    static Uint256 from_progpow(const Hash256& h) { Uint256 r; for (int i = 0; i < 32; ++i) r.data[i] = h.bytes[31 - i]; return r; }
};

struct Uint256Hasher {
    size_t operator()(const Uint256& u) const { return size_t(u.cheap_hash()); }
};

class ArithU256 {
public:
    static constexpr int W = 8;  // 32-bit limbs, little endian
    u32 pn[W];

    ArithU256() { std::memset(pn, 0, sizeof(pn)); }
    ArithU256(u64 v) { std::memset(pn, 0, sizeof(pn)); pn[0] = u32(v); pn[1] = u32(v >> 32); }
    static ArithU256 from_uint256(const Uint256& u) { ArithU256 a; for (int i = 0; i < W; ++i) a.pn[i] = load_le32(u.data + 4 * i); return a; }
    Uint256 to_uint256() const { Uint256 u; for (int i = 0; i < W; ++i) store_le32(u.data + 4 * i, pn[i]); return u; }

    bool is_zero() const { for (u32 x : pn) if (x) return false; return true; }
    int compare(const ArithU256& b) const {
        for (int i = W - 1; i >= 0; --i) {
            if (pn[i] < b.pn[i]) return -1;
            if (pn[i] > b.pn[i]) return 1;
        }
        return 0;
    }
    bool operator==(const ArithU256& b) const { return compare(b) == 0; }
    bool operator!=(const ArithU256& b) const { return compare(b) != 0; }
    bool operator<(const ArithU256& b) const { return compare(b) < 0; }
    bool operator>(const ArithU256& b) const { return compare(b) > 0; }
    bool operator<=(const ArithU256& b) const { return compare(b) <= 0; }
    bool operator>=(const ArithU256& b) const { return compare(b) >= 0; }

    ArithU256 operator~() const { ArithU256 r; for (int i = 0; i < W; ++i) r.pn[i] = ~pn[i]; return r; }
    ArithU256 operator-() const { ArithU256 r = ~*this; r += ArithU256(1); return r; }
    ArithU256& operator+=(const ArithU256& b) {
        u64 carry = 0;
        for (int i = 0; i < W; ++i) { u64 n = carry + pn[i] + b.pn[i]; pn[i] = u32(n); carry = n >> 32; }
        return *this;
    }
    ArithU256& operator-=(const ArithU256& b) { return *this += -b; }
    ArithU256& operator*=(u32 b);
    ArithU256& operator*=(const ArithU256& b);
    ArithU256& operator/=(const ArithU256& b);  // throws on /0 like the reference
    ArithU256& operator<<=(unsigned shift);
    ArithU256& operator>>=(unsigned shift);
    friend ArithU256 operator+(ArithU256 a, const ArithU256& b) { return a += b; }
    friend ArithU256 operator-(ArithU256 a, const ArithU256& b) { return a -= b; }
    friend ArithU256 operator*(ArithU256 a, u32 b) { return a *= b; }
    friend ArithU256 operator*(ArithU256 a, const ArithU256& b) { return a *= b; }
    friend ArithU256 operator/(ArithU256 a, const ArithU256& b) { return a /= b; }
    friend ArithU256 operator<<(ArithU256 a, unsigned s) { return a <<= s; }
    friend ArithU256 operator>>(ArithU256 a, unsigned s) { return a >>= s; }

    unsigned bits() const;
    u64 low64() const { return u64(pn[0]) | (u64(pn[1]) << 32); }
    double getdouble() const;

    ArithU256& set_compact(u32 compact, bool* negative = nullptr, bool* overflow = nullptr);
    u32 get_compact(bool negative = false) const;
    std::string hex() const { return to_uint256().hex(); }
};

}  // namespace nodexa
