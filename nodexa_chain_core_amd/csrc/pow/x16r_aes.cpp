// X16R primitives built on the AES round: Groestl-512, ECHO-512, SHAvite-3-512, Fugue-512.
//
// Parity: sph_groestl512 / sph_echo512 / sph_shavite512 / sph_fugue512 (slots 2, 10,
// 8 and 12 of HashX16R, src/hash.h:335-462). The AES S-box and the GF(2^8) tables
// are derived at start-up (multiplicative inverse + affine map), nothing is stored.
#include "x16r_prims.hpp"

namespace nodexa {

namespace {

u8 xtime(u8 a) { return u8((a << 1) ^ ((a & 0x80) ? 0x1B : 0)); }

u8 gmul(u8 a, u8 b) {
    u8 r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = xtime(a);
        b >>= 1;
    }
    return r;
}

struct Aes {
    u8 sbox[256];
    Aes() {
        for (int x = 0; x < 256; ++x) {
            u8 inv = 0;
            if (x)
                for (int y = 1; y < 256; ++y)
                    if (gmul(u8(x), u8(y)) == 1) { inv = u8(y); break; }
            u8 s = inv;
            for (int k = 1; k <= 4; ++k) s ^= u8((inv << k) | (inv >> (8 - k)));
            sbox[x] = u8(s ^ 0x63);
        }
    }
};

const u8* aes_sbox() {
    static const Aes a;
    return a.sbox;
}

// One AES encryption round on a 16-byte column-major block: SubBytes, ShiftRows,
// MixColumns, AddRoundKey (key may be null = zero key).
void aes_round(u8 s[16], const u8* key) {
    const u8* S = aes_sbox();
    u8 t[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) t[4 * c + r] = S[s[4 * ((c + r) & 3) + r]];
    for (int c = 0; c < 4; ++c) {
        const u8 a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
        s[4 * c + 0] = u8(xtime(a0) ^ xtime(a1) ^ a1 ^ a2 ^ a3);
        s[4 * c + 1] = u8(a0 ^ xtime(a1) ^ xtime(a2) ^ a2 ^ a3);
        s[4 * c + 2] = u8(a0 ^ a1 ^ xtime(a2) ^ xtime(a3) ^ a3);
        s[4 * c + 3] = u8(xtime(a0) ^ a0 ^ a1 ^ a2 ^ xtime(a3));
    }
    if (key)
        for (int i = 0; i < 16; ++i) s[i] ^= key[i];
}

}  // namespace

// ================================================================ Groestl-512
// 8 x 16 byte state (column-major), P1024 / Q1024 with 14 rounds each.
namespace {

void groestl_perm(u8 st[128], bool q) {
    static const int kShiftP[8] = {0, 1, 2, 3, 4, 5, 6, 11};
    static const int kShiftQ[8] = {1, 3, 5, 11, 0, 2, 4, 6};
    static const u8 kMix[8] = {2, 2, 3, 4, 5, 3, 5, 7};
    const u8* S = aes_sbox();
    const int* sh = q ? kShiftQ : kShiftP;
    u8 t[128];
    for (int r = 0; r < 14; ++r) {
        // AddRoundConstant
        for (int j = 0; j < 16; ++j) {
            if (!q) {
                st[8 * j] ^= u8((j << 4) ^ r);
            } else {
                for (int i = 0; i < 7; ++i) st[8 * j + i] ^= 0xFF;
                st[8 * j + 7] ^= u8(0xFF ^ (j << 4) ^ r);
            }
        }
        // SubBytes + ShiftBytes: row i moves left by sh[i] columns
        for (int j = 0; j < 16; ++j)
            for (int i = 0; i < 8; ++i) t[8 * j + i] = S[st[8 * ((j + sh[i]) & 15) + i]];
        // MixBytes: column times circ(2,2,3,4,5,3,5,7)
        for (int j = 0; j < 16; ++j)
            for (int i = 0; i < 8; ++i) {
                u8 v = 0;
                for (int k = 0; k < 8; ++k) v ^= gmul(t[8 * j + k], kMix[(k - i) & 7]);
                st[8 * j + i] = v;
            }
    }
}

void groestl_compress(u8 h[128], const u8 m[128]) {
    u8 p[128], q[128];
    for (int i = 0; i < 128; ++i) { p[i] = h[i] ^ m[i]; q[i] = m[i]; }
    groestl_perm(p, false);
    groestl_perm(q, true);
    for (int i = 0; i < 128; ++i) h[i] ^= p[i] ^ q[i];
}

}  // namespace

Hash512 groestl512(const u8* data, size_t n) {
    u8 h[128] = {0};
    h[126] = 0x02;  // output size 512, 64-bit big-endian at the end of the IV
    u64 blocks = 0;
    for (; n >= 128; n -= 128, data += 128, ++blocks) groestl_compress(h, data);
    u8 buf[256] = {0};
    std::memcpy(buf, data, n);
    buf[n] = 0x80;
    const size_t len = n < 120 ? 128 : 256;
    blocks += len / 128;
    store_be64(buf + len - 8, blocks);
    groestl_compress(h, buf);
    if (len == 256) groestl_compress(h, buf + 128);
    u8 x[128];
    std::memcpy(x, h, 128);
    groestl_perm(x, false);
    Hash512 out;
    for (int i = 0; i < 64; ++i) out.bytes[i] = x[64 + i] ^ h[64 + i];
    return out;
}

// ================================================================ ECHO-512
// 16 x 128-bit words; 1024-bit chaining value, 1024-bit message block, 10 rounds.
namespace {

void echo_compress(u8 v[8][16], const u8 m[128], u64 counter_bits) {
    u8 w[16][16];
    for (int i = 0; i < 8; ++i) std::memcpy(w[i], v[i], 16);
    for (int i = 0; i < 8; ++i) std::memcpy(w[8 + i], m + 16 * i, 16);
    u64 k = counter_bits;
    const u8 salt[16] = {0};
    for (int r = 0; r < 10; ++r) {
        // BIG.SubWords: two AES rounds per word, keys (counter, salt)
        for (int i = 0; i < 16; ++i) {
            u8 key[16] = {0};
            store_le64(key, k);
            ++k;
            aes_round(w[i], key);
            aes_round(w[i], salt);
        }
        // BIG.ShiftRows: word (row i, column j) at index 4j + i; row i rotates by i
        u8 t[16][16];
        for (int j = 0; j < 4; ++j)
            for (int i = 0; i < 4; ++i) std::memcpy(t[4 * j + i], w[4 * ((j + i) & 3) + i], 16);
        // BIG.MixColumns: AES MixColumns across the 4 words of each column, per byte
        for (int j = 0; j < 4; ++j)
            for (int b = 0; b < 16; ++b) {
                const u8 a0 = t[4 * j][b], a1 = t[4 * j + 1][b], a2 = t[4 * j + 2][b], a3 = t[4 * j + 3][b];
                w[4 * j + 0][b] = u8(xtime(a0) ^ xtime(a1) ^ a1 ^ a2 ^ a3);
                w[4 * j + 1][b] = u8(a0 ^ xtime(a1) ^ xtime(a2) ^ a2 ^ a3);
                w[4 * j + 2][b] = u8(a0 ^ a1 ^ xtime(a2) ^ xtime(a3) ^ a3);
                w[4 * j + 3][b] = u8(xtime(a0) ^ a0 ^ a1 ^ a2 ^ xtime(a3));
            }
    }
    // BIG.Final
    for (int i = 0; i < 8; ++i)
        for (int b = 0; b < 16; ++b) v[i][b] ^= m[16 * i + b] ^ w[i][b] ^ w[8 + i][b];
}

}  // namespace

Hash512 echo512(const u8* data, size_t n) {
    u8 v[8][16] = {{0}};
    for (int i = 0; i < 8; ++i) v[i][1] = 0x02;  // 512, 128-bit little-endian
    const u64 total_bits = u64(n) * 8;
    u64 done = 0;
    for (; n >= 128; n -= 128, data += 128) {
        done += 1024;
        echo_compress(v, data, done);
    }
    u8 buf[256] = {0};
    std::memcpy(buf, data, n);
    buf[n] = 0x80;
    const size_t len = n < 110 ? 128 : 256;  // 0x80 + 2-byte size + 16-byte length
    buf[len - 18] = 0x00;
    buf[len - 17] = 0x02;  // 512 as 16-bit little-endian
    store_le64(buf + len - 16, total_bits);
    if (len == 128) {
        echo_compress(v, buf, n ? total_bits : 0);
    } else {
        echo_compress(v, buf, total_bits);
        echo_compress(v, buf + 128, 0);
    }
    Hash512 out;
    for (int i = 0; i < 4; ++i) std::memcpy(out.bytes + 16 * i, v[i], 16);
    return out;
}

Hash512 shavite512(const u8*, size_t) { throw std::runtime_error("shavite512: not implemented"); }
Hash512 fugue512(const u8*, size_t) { throw std::runtime_error("fugue512: not implemented"); }

}  // namespace nodexa
