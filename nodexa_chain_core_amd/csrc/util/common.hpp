// Common fixed-width helpers shared by every native translation unit.
//
// The engine is little-endian only (x86-64 host, gfx950 device); the
// reference's le::/be:: helpers (src/crypto/ethash/lib/ethash/endianness.hpp)
// therefore collapse to identity / byte-swap here.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace nodexa {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
using Bytes = std::vector<u8>;

inline u32 rotl32(u32 x, u32 c) { c &= 31; return c ? (x << c) | (x >> (32 - c)) : x; }
inline u32 rotr32(u32 x, u32 c) { c &= 31; return c ? (x >> c) | (x << (32 - c)) : x; }
inline u64 rotl64(u64 x, u32 c) { c &= 63; return c ? (x << c) | (x >> (64 - c)) : x; }
inline u32 clz32(u32 x) { return x ? u32(__builtin_clz(x)) : 32u; }
inline u32 popc32(u32 x) { return u32(__builtin_popcount(x)); }
inline u32 mulhi32(u32 a, u32 b) { return u32((u64(a) * u64(b)) >> 32); }
inline u32 bswap32(u32 x) { return __builtin_bswap32(x); }
inline u64 bswap64(u64 x) { return __builtin_bswap64(x); }

inline u32 load_le32(const u8* p) { u32 v; std::memcpy(&v, p, 4); return v; }
inline u64 load_le64(const u8* p) { u64 v; std::memcpy(&v, p, 8); return v; }
inline void store_le32(u8* p, u32 v) { std::memcpy(p, &v, 4); }
inline void store_le64(u8* p, u64 v) { std::memcpy(p, &v, 8); }
inline u32 load_be32(const u8* p) { return bswap32(load_le32(p)); }
inline u64 load_be64(const u8* p) { return bswap64(load_le64(p)); }
inline void store_be32(u8* p, u32 v) { store_le32(p, bswap32(v)); }
inline void store_be64(u8* p, u64 v) { store_le64(p, bswap64(v)); }

// FNV-1 / FNV-1a (32-bit) as used by ethash / ProgPoW
// (reference: src/crypto/ethash/lib/ethash/bit_manipulation.h:52-77).
constexpr u32 kFnvPrime = 0x01000193u;
constexpr u32 kFnvOffsetBasis = 0x811c9dc5u;
inline u32 fnv1(u32 u, u32 v) { return (u * kFnvPrime) ^ v; }
inline u32 fnv1a(u32 u, u32 v) { return (u ^ v) * kFnvPrime; }

// Hex helpers. `hex_encode` writes bytes in storage order (the ethash
// to_hex convention); uint256-style reversed display lives in chain/uint256.hpp.
std::string hex_encode(const u8* data, size_t n);
inline std::string hex_encode(const Bytes& b) { return hex_encode(b.data(), b.size()); }
Bytes hex_decode(const std::string& hex);  // throws std::invalid_argument

}  // namespace nodexa
