// Auxiliary hash functions of the node: SHA-1, HMAC-SHA256/512,
// SipHash-2-4 and MurmurHash3.
//
// Parity: CSHA1 (src/crypto/sha1.h), CHMAC_SHA256 / CHMAC_SHA512
// (src/crypto/hmac_sha256.h, hmac_sha512.h), SipHashUint256 / SipHashUint256Extra
// (src/hash.h:317-318, src/hash.cpp:101-256; compact-block short ids and the
// block-index hasher) and MurmurHash3 (src/hash.cpp:24; bloom filters). Written
// from FIPS 180-4, RFC 2104, Aumasson-Bernstein 2012 and Appleby's MurmurHash3.
#pragma once

#include "../util/common.hpp"

namespace nodexa {

void sha1(const u8* data, size_t n, u8 out[20]);
void hmac_sha256(const u8* key, size_t klen, const u8* msg, size_t mlen, u8 out[32]);
void hmac_sha512(const u8* key, size_t klen, const u8* msg, size_t mlen, u8 out[64]);

u64 siphash24(u64 k0, u64 k1, const u8* data, size_t n);
// SipHash-2-4 of a uint256 (32 storage bytes), and of uint256 || le32(extra).
u64 siphash_uint256(u64 k0, u64 k1, const u8 val[32]);
u64 siphash_uint256_extra(u64 k0, u64 k1, const u8 val[32], u32 extra);

u32 murmur3_32(u32 seed, const u8* data, size_t n);

}  // namespace nodexa
