// BLAKE2b (RFC 7693) with a parameter block (digest length, personalization).
// Used by Equihash(200,9): digest 50 bytes, personal = "ZcashPoW"||le32(n)||le32(k).
#pragma once

#include "../util/common.hpp"

namespace nodexa {

struct Blake2b {
    u64 h[8];
    u64 t[2] = {0, 0};
    u8 buf[128];
    size_t buflen = 0;
    size_t outlen = 64;

    // personal: 16 bytes or nullptr.
    Blake2b(size_t outlen, const u8* personal = nullptr);
    Blake2b& update(const u8* data, size_t n);
    void final(u8* out);
    static void compress(u64 h[8], const u8 block[128], u64 t0, u64 t1, bool last);
};

void blake2b(const u8* data, size_t n, u8* out, size_t outlen);

}  // namespace nodexa
