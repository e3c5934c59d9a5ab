// Hash functions the reference links into its node but never calls from consensus:
// HAVAL (src/algo/haval.c, haval_helper.c: sph_haval{128,160,192,224,256}_{3,4,5}), GOST
// Streebog (src/algo/gost_streebog.c) and the
// Lyra2 password hash over its reduced-BLAKE2b sponge (src/algo/lyra2.cpp LYRA2 / LYRA2_old,
// src/algo/sponge.cpp). Written from the HAVAL paper (Zheng, Pieprzyk, Seberry 1992) and the
// Lyra2 reference description; round constants are derived, not tabulated (see the .cpp).
#pragma once

#include <vector>

#include "../util/common.hpp"

namespace nodexa {

// HAVAL with `passes` in {3,4,5} and `out_bits` in {128,160,192,224,256}; returns out_bits/8 bytes.
std::vector<u8> haval_hash(const u8* data, size_t n, int passes, int out_bits);

// LYRA2(K, kLen, pwd, salt, timeCost, nRows, nCols). `old_absorb` reproduces LYRA2_old, which
// steps its input pointer by 64 words instead of 8 between the 64-byte input blocks (the two differ
// only when pwd + salt + 48 bytes > 64). nRows must be a power of two >= 4 (the reference's
// setup-phase window arithmetic assumes it; 2 rows overrun its matrix); returns kLen bytes, or empty on invalid parameters.
// GOST R 34.11-2012 (Streebog) with the reference's byte conventions (src/algo/gost_streebog.c:
// sph_gost256 / sph_gost512, one-shot); out_bits 256 or 512.
std::vector<u8> gost_streebog(const u8* data, size_t n, int out_bits);

std::vector<u8> lyra2_hash(const u8* pwd, size_t pwdlen, const u8* salt, size_t saltlen, u64 klen, u64 time_cost,
                           u64 n_rows, u64 n_cols, bool old_absorb = false);

}  // namespace nodexa
