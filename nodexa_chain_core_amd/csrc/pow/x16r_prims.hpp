// The sixteen 512-bit primitives of X16R / X16RV2 (+ Tiger-192 for X16RV2).
//
// Parity: the sph_* family the reference links for HashX16R / HashX16RV2
// (src/hash.h:335-605, src/algo/*.c, src/algo/tiger.cpp). Every primitive here
// is written from its published specification (SHA-3 round-2/3 submissions,
// Whirlpool ISO/IEC 10118-3, Tiger 1995) as a plain one-shot function over a
// byte string; tests/test_x16r.py pins each against golden digests produced by
// compiling the reference's own sources (tools/ref_x16r_vectors.sh).
#pragma once

#include "../crypto/keccak.hpp"
#include "../util/common.hpp"

namespace nodexa {

Hash512 blake512(const u8* data, size_t n);       // slot 0   (x16r.cpp)
Hash512 bmw512(const u8* data, size_t n);         // slot 1   (x16r_arx.cpp)
Hash512 groestl512(const u8* data, size_t n);     // slot 2   (x16r_aes.cpp)
Hash512 jh512(const u8* data, size_t n);          // slot 3   (x16r_bitslice.cpp)
/* keccak512 */                                   // slot 4   (crypto/keccak.cpp)
Hash512 skein512(const u8* data, size_t n);       // slot 5   (x16r_arx.cpp)
Hash512 luffa512(const u8* data, size_t n);       // slot 6   (x16r_bitslice.cpp)
Hash512 cubehash512(const u8* data, size_t n);    // slot 7   (x16r_arx.cpp)
Hash512 shavite512(const u8* data, size_t n);     // slot 8   (x16r_aes.cpp)
Hash512 simd512(const u8* data, size_t n);        // slot 9   (x16r_simd.cpp)
Hash512 echo512(const u8* data, size_t n);        // slot 10  (x16r_aes.cpp)
Hash512 hamsi512(const u8* data, size_t n);       // slot 11  (x16r_bitslice.cpp)
Hash512 fugue512(const u8* data, size_t n);       // slot 12  (x16r_aes.cpp)
Hash512 shabal512(const u8* data, size_t n);      // slot 13  (x16r_arx.cpp)
Hash512 whirlpool512(const u8* data, size_t n);   // slot 14  (x16r_sbox64.cpp)
Hash512 sha512_hash(const u8* data, size_t n);    // slot 15  (x16r.cpp)
Hash512 tiger192_padded(const u8* data, size_t n);  // X16RV2 pre-hash: 24 bytes + 40 zero bytes (x16r_sbox64.cpp)

}  // namespace nodexa
