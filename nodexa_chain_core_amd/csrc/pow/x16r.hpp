// X16R / X16RV2 legacy proof-of-work (pre-KawPow headers).
//
// Parity: HashX16R / HashX16RV2 (src/hash.h:335-605), GetHashSelection
// (src/hash.h:320-327: nibble 48+i of hashPrevBlock picks algorithm i).
// Algorithm slots: 0 blake512, 1 bmw512, 2 groestl512, 3 jh512, 4 keccak512,
// 5 skein512, 6 luffa512, 7 cubehash512, 8 shavite512, 9 simd512, 10 echo512,
// 11 hamsi512, 12 fugue512, 13 shabal512, 14 whirlpool, 15 sha512; X16RV2
// prefixes slots 4, 6 and 15 with Tiger-192 (zero-extended to 64 bytes).
// The primitives are written from their published specifications.
#pragma once

#include "../crypto/keccak.hpp"

namespace nodexa {

// out = trim256(X16R(data)) in uint256 storage order; prev_le = hashPrevBlock storage bytes.
void x16r_hash(const u8* data, size_t n, const u8 prev_le[32], bool v2, u8 out[32]);
// One 512-bit primitive (slot 0..15), or 16 = Tiger-192 zero-padded to 64 bytes.
Hash512 x16r_single(int algo, const u8* data, size_t n);
// True when every slot of the selection is implemented in this build.
bool x16r_slot_available(int algo);
int x16r_selection(const u8 prev_le[32], int index);

// Legacy-header nonce search (32-bit nNonce at byte 76 of the 80-byte header;
// hashPrevBlock at bytes 4..35 drives the algorithm order). Lowest nonce in
// [start, start + count) whose hash <= target (little-endian uint256 storage).
struct X16rSearchResult {
    bool found = false;
    u32 nonce = 0;
    u64 hashes = 0;
    u8 hash[32] = {0};
};
X16rSearchResult x16r_search(const u8 header80[80], bool v2, const u8 target_le[32], u32 start, u64 count,
                             int threads);

// Individual primitives: x16r_prims.hpp.

}  // namespace nodexa
