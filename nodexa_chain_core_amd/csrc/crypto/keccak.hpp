// Keccak permutations and the original-Keccak sponge (0x01 .. 0x80 padding).
//
// Parity: keccakf1600 (src/crypto/ethash/lib/keccak/keccakf1600.c:40),
// keccakf800 (src/crypto/ethash/lib/keccak/keccakf800.c:38), keccak256/512
// (src/crypto/ethash/lib/keccak/keccak.c:46-127). Written from the Keccak
// reference specification; the same permutation is re-expressed for the GPU in
// hip/kernels/keccak_device.hpp.
#pragma once

#include "../util/common.hpp"

namespace nodexa {

struct Hash256 {
    union { u8 bytes[32]; u32 w32[8]; u64 w64[4]; };
    Hash256() { std::memset(bytes, 0, 32); }
    bool operator==(const Hash256& o) const { return std::memcmp(bytes, o.bytes, 32) == 0; }
    bool operator!=(const Hash256& o) const { return !(*this == o); }
};
struct Hash512 {
    union { u8 bytes[64]; u32 w32[16]; u64 w64[8]; };
    Hash512() { std::memset(bytes, 0, 64); }
    bool operator==(const Hash512& o) const { return std::memcmp(bytes, o.bytes, 64) == 0; }
};

extern const u64 kKeccakRoundConstants[24];

void keccakf1600(u64 st[25]);
void keccakf800(u32 st[25]);  // 22 rounds

// Original Keccak (not SHA-3) with 256/512-bit output.
Hash256 keccak256(const u8* data, size_t n);
Hash512 keccak512(const u8* data, size_t n);
inline Hash256 keccak256(const Hash256& h) { return keccak256(h.bytes, 32); }
inline Hash512 keccak512(const Hash512& h) { return keccak512(h.bytes, 64); }

// Big-endian 256-bit comparison a <= b (ethash is_less_or_equal,
// src/crypto/ethash/lib/ethash/ethash-internal.hpp:32-42).
bool hash_le(const Hash256& a, const Hash256& b);

Hash256 hash256_from_hex(const std::string& hex);  // storage order
std::string hash256_to_hex(const Hash256& h);

}  // namespace nodexa
