// SHA-256 / double-SHA-256 (FIPS 180-4).
//
// Parity: CSHA256 (src/crypto/sha256.h:16), CHash256 / SerializeHash
// (src/hash.h:49,274). Block-header hashing for KawPow (CKAWPOWInput,
// src/primitives/block.h:213-233) and merkle roots use sha256d.
#pragma once

#include "../util/common.hpp"

namespace nodexa {

class Sha256 {
public:
    Sha256() { reset(); }
    Sha256& reset();
    Sha256& write(const u8* data, size_t n);
    void finalize(u8 out[32]);

    static void compress(u32 state[8], const u8 block[64]);                   // portable
    static void compress_blocks(u32 state[8], const u8* data, size_t blocks);  // SHA-NI when present

private:
    u32 s_[8];
    u8 buf_[64];
    u64 bytes_ = 0;
};

void sha256(const u8* data, size_t n, u8 out[32]);
void sha256d(const u8* data, size_t n, u8 out[32]);
// sha256d of exactly two concatenated 32-byte nodes (merkle inner node).
void sha256d_64(const u8 left[32], const u8 right[32], u8 out[32]);

}  // namespace nodexa
