// X16R primitives over 4-bit / bit-sliced state: JH-512, Luffa-512, Hamsi-512.
//
// Parity: sph_jh512 / sph_luffa512 / sph_hamsi512 (slots 3, 6 and 11 of HashX16R,
// src/hash.h:335-462). Written from the SHA-3 round-3 / round-2 specifications;
// round constants are generated, not stored, wherever the spec defines them
// procedurally (JH: R6 iterated from the fractional bits of sqrt(2)).
#include "x16r_prims.hpp"

namespace nodexa {

// ================================================================ JH-512 (42 rounds)
// Element form of E8: 256 4-bit elements; R8 = S-box layer (round-constant bit picks
// S0/S1), MDS layer L on element pairs, permutation P8 = phi . P' . pi. The round
// constant itself is advanced by R6 with constant zero.
namespace {

const u8 kJhS[2][16] = {{9, 0, 4, 11, 13, 12, 3, 15, 1, 10, 2, 6, 7, 5, 8, 14},
                        {3, 12, 6, 13, 5, 7, 1, 9, 15, 2, 0, 4, 11, 10, 14, 8}};

inline u8 jh_mul2(u8 a) { return u8(((a << 1) ^ (a >> 3) ^ ((a >> 2) & 2)) & 0xF); }

inline void jh_L(u8& a, u8& b) {
    b ^= jh_mul2(a);
    a ^= jh_mul2(b);
}

// One round of R_d over `n` = 2^d elements (d = 8 for the state, 6 for the constant).
void jh_round(u8* x, int n, const u8* sel) {
    u8 t[256];
    for (int i = 0; i < n; ++i) t[i] = kJhS[sel ? sel[i] : 0][x[i]];
    for (int i = 0; i < n; i += 2) jh_L(t[i], t[i + 1]);
    for (int i = 0; i < n; i += 4) std::swap(t[i + 2], t[i + 3]);  // pi
    for (int i = 0; i < n / 2; ++i) {                              // P'
        x[i] = t[2 * i];
        x[i + n / 2] = t[2 * i + 1];
    }
    for (int i = n / 2; i < n; i += 2) std::swap(x[i], x[i + 1]);  // phi
}

struct JhConstants {
    u8 sel[42][256];  // per round, per element: S-box selector bit
    JhConstants() {
        static const char* c0 = "6a09e667f3bcc908b2fb1366ea957d3e3adec17512775099da2f590b0667322a";
        u8 rc[64];
        for (int i = 0; i < 64; ++i) {
            const char c = c0[i];
            rc[i] = u8(c <= '9' ? c - '0' : c - 'a' + 10);
        }
        for (int r = 0; r < 42; ++r) {
            for (int i = 0; i < 256; ++i) sel[r][i] = (rc[i >> 2] >> (3 - (i & 3))) & 1;
            jh_round(rc, 64, nullptr);
        }
    }
};

void jh_e8(u8 H[128]) {
    static const JhConstants k;
    auto bit = [&](int i) { return (H[i >> 3] >> (7 - (i & 7))) & 1; };
    u8 tmp[256], A[256];
    for (int i = 0; i < 256; ++i)
        tmp[i] = u8((bit(i) << 3) | (bit(i + 256) << 2) | (bit(i + 512) << 1) | bit(i + 768));
    for (int i = 0; i < 128; ++i) {
        A[2 * i] = tmp[i];
        A[2 * i + 1] = tmp[i + 128];
    }
    for (int r = 0; r < 42; ++r) jh_round(A, 256, k.sel[r]);
    for (int i = 0; i < 128; ++i) {
        tmp[i] = A[2 * i];
        tmp[i + 128] = A[2 * i + 1];
    }
    std::memset(H, 0, 128);
    for (int i = 0; i < 256; ++i)
        for (int b = 0; b < 4; ++b) {
            const int pos = i + 256 * b;
            H[pos >> 3] |= u8(((tmp[i] >> (3 - b)) & 1) << (7 - (pos & 7)));
        }
}

void jh_f8(u8 H[128], const u8 m[64]) {
    for (int i = 0; i < 64; ++i) H[i] ^= m[i];
    jh_e8(H);
    for (int i = 0; i < 64; ++i) H[64 + i] ^= m[i];
}

struct JhIV {
    u8 H[128] = {0};
    JhIV() {
        H[0] = 0x02;  // hash bit length 512, 16-bit big-endian
        const u8 zero[64] = {0};
        jh_f8(H, zero);
    }
};

}  // namespace

Hash512 jh512(const u8* data, size_t n) {
    static const JhIV iv;
    u8 H[128];
    std::memcpy(H, iv.H, 128);
    const u64 bits = u64(n) * 8;
    for (; n >= 64; n -= 64, data += 64) jh_f8(H, data);
    // 0x80, zeros, 128-bit big-endian length; always at least one extra 512-bit block
    u8 buf[128] = {0};
    std::memcpy(buf, data, n);
    buf[n] = 0x80;
    const size_t len = n == 0 ? 64 : 128;
    store_be64(buf + len - 8, bits);
    jh_f8(H, buf);
    if (len == 128) jh_f8(H, buf + 64);
    Hash512 out;
    std::memcpy(out.bytes, H + 64, 64);
    return out;
}

Hash512 luffa512(const u8*, size_t) { throw std::runtime_error("luffa512: not implemented"); }
Hash512 hamsi512(const u8*, size_t) { throw std::runtime_error("hamsi512: not implemented"); }

}  // namespace nodexa
