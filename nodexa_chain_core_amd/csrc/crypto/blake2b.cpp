#include "blake2b.hpp"

namespace nodexa {

namespace {
const u64 kIV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                    0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
const u8 kSigma[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
inline u64 rotr(u64 x, int n) { return (x >> n) | (x << (64 - n)); }
}  // namespace

void Blake2b::compress(u64 h[8], const u8 block[128], u64 t0, u64 t1, bool last) {
    u64 m[16], v[16];
    for (int i = 0; i < 16; ++i) m[i] = load_le64(block + 8 * i);
    for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = kIV[i]; }
    v[12] ^= t0;
    v[13] ^= t1;
    if (last) v[14] = ~v[14];
    auto G = [&](int a, int b, int c, int d, u64 x, u64 y) {
        v[a] = v[a] + v[b] + x; v[d] = rotr(v[d] ^ v[a], 32);
        v[c] = v[c] + v[d];     v[b] = rotr(v[b] ^ v[c], 24);
        v[a] = v[a] + v[b] + y; v[d] = rotr(v[d] ^ v[a], 16);
        v[c] = v[c] + v[d];     v[b] = rotr(v[b] ^ v[c], 63);
    };
    for (int r = 0; r < 12; ++r) {
        const u8* s = kSigma[r];
        G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

Blake2b::Blake2b(size_t out, const u8* personal) : outlen(out) {
    u8 param[64] = {0};
    param[0] = u8(out);
    param[2] = 1;  // fanout
    param[3] = 1;  // depth
    if (personal) std::memcpy(param + 48, personal, 16);
    for (int i = 0; i < 8; ++i) h[i] = kIV[i] ^ load_le64(param + 8 * i);
}

Blake2b& Blake2b::update(const u8* data, size_t n) {
    while (n > 0) {
        if (buflen == 128) {  // keep the last block for final()
            t[0] += 128;
            if (t[0] < 128) ++t[1];
            compress(h, buf, t[0], t[1], false);
            buflen = 0;
        }
        const size_t take = std::min(n, 128 - buflen);
        std::memcpy(buf + buflen, data, take);
        buflen += take;
        data += take;
        n -= take;
    }
    return *this;
}

void Blake2b::final(u8* out) {
    t[0] += buflen;
    if (t[0] < buflen) ++t[1];
    std::memset(buf + buflen, 0, 128 - buflen);
    compress(h, buf, t[0], t[1], true);
    u8 full[64];
    for (int i = 0; i < 8; ++i) store_le64(full + 8 * i, h[i]);
    std::memcpy(out, full, outlen);
}

void blake2b(const u8* data, size_t n, u8* out, size_t outlen) {
    Blake2b s(outlen);
    s.update(data, n).final(out);
}

}  // namespace nodexa
