#include "sha256.hpp"

#include <immintrin.h>

namespace nodexa {

namespace {
constexpr u32 K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
constexpr u32 H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                       0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
}  // namespace

// x86 SHA extensions path (runtime-dispatched; the reference picks its SSE4 transform
// the same way, src/crypto/sha256.cpp:187-189).
__attribute__((target("sha,sse4.1"))) static void compress_shani(u32 st[8], const u8* data, size_t blocks) {
    const __m128i mask = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i tmp = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(st)), 0xB1);
    __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(st + 4)), 0x1B);
    __m128i s0 = _mm_alignr_epi8(tmp, s1, 8);  // ABEF
    s1 = _mm_blend_epi16(s1, tmp, 0xF0);      // CDGH
    for (; blocks; --blocks, data += 64) {
        const __m128i abef = s0, cdgh = s1;
        __m128i m[4];
        for (int g = 0; g < 16; ++g) {
            if (g < 4) {
                m[g] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(data + 16 * g)), mask);
            } else {  // W[4g..4g+3] from groups g-4 .. g-1 held in m[g&3], m[(g+1)&3], m[(g+2)&3], m[(g+3)&3]
                const __m128i t = _mm_add_epi32(_mm_sha256msg1_epu32(m[g & 3], m[(g + 1) & 3]),
                                                _mm_alignr_epi8(m[(g + 3) & 3], m[(g + 2) & 3], 4));
                m[g & 3] = _mm_sha256msg2_epu32(t, m[(g + 3) & 3]);
            }
            const __m128i wk = _mm_add_epi32(m[g & 3], _mm_loadu_si128(reinterpret_cast<const __m128i*>(K + 4 * g)));
            s1 = _mm_sha256rnds2_epu32(s1, s0, wk);
            s0 = _mm_sha256rnds2_epu32(s0, s1, _mm_shuffle_epi32(wk, 0x0E));
        }
        s0 = _mm_add_epi32(s0, abef);
        s1 = _mm_add_epi32(s1, cdgh);
    }
    tmp = _mm_shuffle_epi32(s0, 0x1B);     // FEBA
    s1 = _mm_shuffle_epi32(s1, 0xB1);      // DCHG
    s0 = _mm_blend_epi16(tmp, s1, 0xF0);   // DCBA
    s1 = _mm_alignr_epi8(s1, tmp, 8);      // HGFE
    _mm_storeu_si128(reinterpret_cast<__m128i*>(st), s0);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(st + 4), s1);
}

static bool have_shani() {
    static const bool ok = __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
    return ok;
}

void Sha256::compress_blocks(u32 s[8], const u8* data, size_t blocks) {
    if (have_shani()) {
        compress_shani(s, data, blocks);
        return;
    }
    for (; blocks; --blocks, data += 64) compress(s, data);
}

void Sha256::compress(u32 s[8], const u8 block[64]) {
    u32 w[64];
    for (int i = 0; i < 16; ++i) w[i] = load_be32(block + 4 * i);
    for (int i = 16; i < 64; ++i) {
        const u32 s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        const u32 s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    u32 a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
    for (int i = 0; i < 64; ++i) {
        const u32 S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
        const u32 ch = (e & f) ^ (~e & g);
        const u32 t1 = h + S1 + ch + K[i] + w[i];
        const u32 S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
        const u32 maj = (a & b) ^ (a & c) ^ (b & c);
        const u32 t2 = S0 + maj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

Sha256& Sha256::reset() {
    std::memcpy(s_, H0, sizeof(s_));
    bytes_ = 0;
    return *this;
}

Sha256& Sha256::write(const u8* data, size_t n) {
    size_t fill = bytes_ % 64;
    bytes_ += n;
    if (fill) {
        const size_t take = std::min<size_t>(64 - fill, n);
        std::memcpy(buf_ + fill, data, take);
        data += take;
        n -= take;
        if (fill + take < 64) return *this;
        compress_blocks(s_, buf_, 1);
    }
    if (n >= 64) {
        compress_blocks(s_, data, n / 64);
        data += n / 64 * 64;
        n %= 64;
    }
    if (n) std::memcpy(buf_, data, n);
    return *this;
}

void Sha256::finalize(u8 out[32]) {
    const u64 bits = bytes_ * 8;
    u8 pad[72] = {0x80};
    const size_t fill = bytes_ % 64;
    const size_t padlen = (fill < 56) ? (56 - fill) : (120 - fill);
    write(pad, padlen);
    u8 len[8];
    store_be64(len, bits);
    write(len, 8);
    for (int i = 0; i < 8; ++i) store_be32(out + 4 * i, s_[i]);
}

void sha256(const u8* data, size_t n, u8 out[32]) { Sha256().write(data, n).finalize(out); }

void sha256d(const u8* data, size_t n, u8 out[32]) {
    u8 tmp[32];
    sha256(data, n, tmp);
    sha256(tmp, 32, out);
}

void sha256d_64(const u8 left[32], const u8 right[32], u8 out[32]) {
    u8 buf[64];
    std::memcpy(buf, left, 32);
    std::memcpy(buf + 32, right, 32);
    sha256d(buf, 64, out);
}

}  // namespace nodexa
