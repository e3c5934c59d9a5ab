#include "hashes.hpp"

#include <immintrin.h>

#include "../pow/x16r_prims.hpp"
#include "sha256.hpp"

namespace nodexa {

// ---------------------------------------------------------------- SHA-1 (FIPS 180-4 §6.1)
namespace {
void sha1_block(u32 h[5], const u8* p) {
    u32 w[80];
    for (int i = 0; i < 16; ++i) w[i] = load_be32(p + 4 * i);
    for (int i = 16; i < 80; ++i) w[i] = rotl32(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    u32 a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int i = 0; i < 80; ++i) {
        u32 f, k;
        if (i < 20) { f = (b & c) | (~b & d); k = 0x5A827999u; }
        else if (i < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1u; }
        else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDCu; }
        else { f = b ^ c ^ d; k = 0xCA62C1D6u; }
        const u32 t = rotl32(a, 5) + f + e + k + w[i];
        e = d; d = c; c = rotl32(b, 30); b = a; a = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}
__attribute__((target("sha,sse4.1"))) void sha1_shani(u32 h[5], const u8* data, size_t blocks) {
    const __m128i mask = _mm_set_epi64x(0x0001020304050607ULL, 0x08090a0b0c0d0e0fULL);
    __m128i abcd = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(h)), 0x1B);
    __m128i e0 = _mm_set_epi32(int(h[4]), 0, 0, 0);
    for (; blocks; --blocks, data += 64) {
        const __m128i abcd_save = abcd, e_save = e0;
        __m128i m[4], prev = abcd, e = e0;
        for (int g = 0; g < 20; ++g) {
            if (g < 4)
                m[g] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(data + 16 * g)), mask);
            else  // W[4g..4g+3] from groups g-4 (m[g&3]), g-3, g-2, g-1
                m[g & 3] = _mm_sha1msg2_epu32(
                    _mm_xor_si128(_mm_sha1msg1_epu32(m[g & 3], m[(g + 1) & 3]), m[(g + 2) & 3]), m[(g + 3) & 3]);
            e = g == 0 ? _mm_add_epi32(e0, m[0]) : _mm_sha1nexte_epu32(prev, m[g & 3]);
            prev = abcd;
            switch (g / 5) {  // rnds4 takes the round function as an immediate
                case 0: abcd = _mm_sha1rnds4_epu32(abcd, e, 0); break;
                case 1: abcd = _mm_sha1rnds4_epu32(abcd, e, 1); break;
                case 2: abcd = _mm_sha1rnds4_epu32(abcd, e, 2); break;
                default: abcd = _mm_sha1rnds4_epu32(abcd, e, 3); break;
            }
        }
        e0 = _mm_sha1nexte_epu32(prev, e_save);
        abcd = _mm_add_epi32(abcd, abcd_save);
    }
    _mm_storeu_si128(reinterpret_cast<__m128i*>(h), _mm_shuffle_epi32(abcd, 0x1B));
    h[4] = u32(_mm_extract_epi32(e0, 3));
}

void sha1_blocks(u32 h[5], const u8* data, size_t blocks) {
    static const bool shani = __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
    if (shani) {
        sha1_shani(h, data, blocks);
        return;
    }
    for (; blocks; --blocks, data += 64) sha1_block(h, data);
}
}  // namespace

void sha1(const u8* data, size_t n, u8 out[20]) {
    u32 h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    const u64 bits = u64(n) * 8;
    sha1_blocks(h, data, n / 64);
    data += n / 64 * 64;
    n %= 64;
    u8 buf[128] = {0};
    if (n) std::memcpy(buf, data, n);  // data may be null when n == 0
    buf[n] = 0x80;
    const size_t len = n < 56 ? 64 : 128;
    store_be64(buf + len - 8, bits);
    sha1_blocks(h, buf, len / 64);
    for (int i = 0; i < 5; ++i) store_be32(out + 4 * i, h[i]);
}

// ---------------------------------------------------------------- HMAC (RFC 2104)
void hmac_sha256(const u8* key, size_t klen, const u8* msg, size_t mlen, u8 out[32]) {
    u8 k[64] = {0};
    if (klen > 64) sha256(key, klen, k);
    else std::memcpy(k, key, klen);
    u8 pad[64], inner[32];
    for (int i = 0; i < 64; ++i) pad[i] = k[i] ^ 0x36;
    Sha256().write(pad, 64).write(msg, mlen).finalize(inner);
    for (int i = 0; i < 64; ++i) pad[i] = k[i] ^ 0x5c;
    Sha256().write(pad, 64).write(inner, 32).finalize(out);
}

void hmac_sha512(const u8* key, size_t klen, const u8* msg, size_t mlen, u8 out[64]) {
    u8 k[128] = {0};
    if (klen > 128) std::memcpy(k, sha512_hash(key, klen).bytes, 64);
    else std::memcpy(k, key, klen);
    Bytes buf(128 + mlen);
    for (int i = 0; i < 128; ++i) buf[i] = k[i] ^ 0x36;
    std::memcpy(buf.data() + 128, msg, mlen);
    const Hash512 inner = sha512_hash(buf.data(), buf.size());
    u8 outer[192];
    for (int i = 0; i < 128; ++i) outer[i] = k[i] ^ 0x5c;
    std::memcpy(outer + 128, inner.bytes, 64);
    std::memcpy(out, sha512_hash(outer, 192).bytes, 64);
}

// ---------------------------------------------------------------- SipHash-2-4
u64 siphash24(u64 k0, u64 k1, const u8* data, size_t n) {
    u64 v0 = 0x736f6d6570736575ULL ^ k0, v1 = 0x646f72616e646f6dULL ^ k1;
    u64 v2 = 0x6c7967656e657261ULL ^ k0, v3 = 0x7465646279746573ULL ^ k1;
    auto round = [&] {
        v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0; v0 = rotl64(v0, 32);
        v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;
        v0 += v3; v3 = rotl64(v3, 21); v3 ^= v0;
        v2 += v1; v1 = rotl64(v1, 17); v1 ^= v2; v2 = rotl64(v2, 32);
    };
    auto absorb = [&](u64 m) {
        v3 ^= m;
        round();
        round();
        v0 ^= m;
    };
    const size_t total = n;
    for (; n >= 8; n -= 8, data += 8) absorb(load_le64(data));
    u64 last = u64(total & 0xFF) << 56;
    for (size_t i = 0; i < n; ++i) last |= u64(data[i]) << (8 * i);
    absorb(last);
    v2 ^= 0xFF;
    round(); round(); round(); round();
    return v0 ^ v1 ^ v2 ^ v3;
}

u64 siphash_uint256(u64 k0, u64 k1, const u8 val[32]) { return siphash24(k0, k1, val, 32); }

u64 siphash_uint256_extra(u64 k0, u64 k1, const u8 val[32], u32 extra) {
    u8 buf[36];
    std::memcpy(buf, val, 32);
    store_le32(buf + 32, extra);
    return siphash24(k0, k1, buf, 36);
}

// ---------------------------------------------------------------- MurmurHash3 x86_32
u32 murmur3_32(u32 seed, const u8* data, size_t n) {
    const u32 c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    u32 h = seed;
    const size_t blocks = n / 4;
    for (size_t i = 0; i < blocks; ++i) {
        u32 k = load_le32(data + 4 * i);
        k *= c1; k = rotl32(k, 15); k *= c2;
        h ^= k; h = rotl32(h, 13); h = h * 5 + 0xe6546b64u;
    }
    const u8* tail = data + 4 * blocks;
    u32 k = 0;
    switch (n & 3) {
        case 3: k ^= u32(tail[2]) << 16; [[fallthrough]];
        case 2: k ^= u32(tail[1]) << 8; [[fallthrough]];
        case 1: k ^= tail[0]; k *= c1; k = rotl32(k, 15); k *= c2; h ^= k;
    }
    h ^= u32(n);
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

}  // namespace nodexa
