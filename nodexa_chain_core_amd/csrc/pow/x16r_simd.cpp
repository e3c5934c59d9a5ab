// X16R slot 9: SIMD-512 (Leurent, Bouillaguet, Fouque — SHA-3 round 2, v1.1).
//
// Parity: sph_simd512 as linked by HashX16R (src/hash.h:335-462). Written from
// the specification: the 1024-bit message block is expanded by a 256-point
// number-theoretic transform over Z_257 (root 41), tweaked with X^255 (and
// X^253 for the final block), lifted to 16-bit words by x185 / x233 and paired
// into 32 x 8 message words; four rounds of eight Feistel steps over four
// 8-word registers (IF for the first half of a round, MAJ for the second),
// rotations (r, s) chained per round, lane permutations n -> n ^ c, and a
// four-step feed-forward of the incoming chaining value. The transform is a radix-2 NTT
// (256 points, 8 stages).
#include "x16r_prims.hpp"

namespace nodexa {

namespace {

struct SimdTables {
    int pw[256];       // 41^k mod 257
    int yoff_n[256];   // beta^(255 i)
    int yoff_f[256];   // beta^(255 i) + beta^(253 i)
    SimdTables() {
        pw[0] = 1;
        for (int k = 1; k < 256; ++k) pw[k] = pw[k - 1] * 41 % 257;
        for (int i = 0; i < 256; ++i) {
            yoff_n[i] = pw[(255 * i) % 256];
            yoff_f[i] = (pw[(255 * i) % 256] + pw[(253 * i) % 256]) % 257;
        }
    }
};

const SimdTables& simd_tables() {
    static const SimdTables t;
    return t;
}

inline u32 simd_if(u32 x, u32 y, u32 z) { return ((y ^ z) & x) ^ z; }
inline u32 simd_maj(u32 x, u32 y, u32 z) { return (x & y) | ((x | y) & z); }

struct SimdState {
    u32 A[8], B[8], C[8], D[8];

    // One step: w = 8 message words, f = 0 (IF) / 1 (MAJ), rotations r, s, permutation n ^ pc.
    void step(const u32 w[8], int f, int r, int s, int pc) {
        u32 tA[8];
        for (int n = 0; n < 8; ++n) tA[n] = rotl32(A[n], r);
        for (int n = 0; n < 8; ++n) {
            const u32 fv = f ? simd_maj(A[n], B[n], C[n]) : simd_if(A[n], B[n], C[n]);
            const u32 tt = D[n] + w[n] + fv;
            A[n] = rotl32(tt, s) + tA[n ^ pc];
            D[n] = C[n];
            C[n] = B[n];
            B[n] = tA[n];
        }
    }
};

// y_i = sum_j blk[j] 41^(ij) mod 257 (the 128 bytes zero-extended to 256 points): radix-2
// decimation-in-time NTT, bit-reversed input, 8 stages of 128 butterflies; then the X^255 (and, for
// the final block, X^253) tweak and the centred lift to [-128, 128]
void simd_expand(const u8 blk[128], bool last, int q[256]) {
    const SimdTables& T = simd_tables();
    for (int j = 0; j < 256; ++j) {
        int r = 0;
        for (int b = 0; b < 8; ++b) r |= ((j >> b) & 1) << (7 - b);
        q[r] = j < 128 ? int(blk[j]) : 0;
    }
    for (int len = 2; len <= 256; len <<= 1) {
        const int half = len / 2, stride = 256 / len;
        for (int i = 0; i < 256; i += len)
            for (int k = 0; k < half; ++k) {
                const int u = q[i + k], v = q[i + k + half] * T.pw[stride * k] % 257;
                q[i + k] = (u + v) % 257;
                q[i + k + half] = (u - v + 257) % 257;
            }
    }
    const int* yoff = last ? T.yoff_f : T.yoff_n;
    for (int i = 0; i < 256; ++i) {
        const int acc = (q[i] + yoff[i]) % 257;
        q[i] = acc <= 128 ? acc : acc - 257;
    }
}

// The final block of a 64- or 80-byte message (every X16R input) is its bit length and zeros:
// its expansion is a constant, computed once (and emitted for the GPU, tools/x16r_gen_tables.cpp).
struct SimdFinal {
    int q64[256], q80[256];
    SimdFinal() {
        u8 blk[128] = {0};
        store_le64(blk, 64 * 8);
        simd_expand(blk, true, q64);
        store_le64(blk, 80 * 8);
        simd_expand(blk, true, q80);
    }
};

const SimdFinal& simd_final() {
    static const SimdFinal f;
    return f;
}

void simd_rounds(u32 state[32], const u8 blk[128], const int q[256]) {
    // message words: 4 rounds x 8 steps x 8 lanes, from q pairs lifted by 185 / 233
    auto inner = [](int lo, int hi, int mm) { return (u32(lo * mm) & 0xFFFFu) + (u32(hi * mm) << 16); };
    static const int kSb[4][8] = {{4, 6, 0, 2, 7, 5, 3, 1}, {15, 11, 12, 8, 9, 13, 10, 14},
                                  {17, 18, 23, 20, 22, 21, 16, 19}, {30, 24, 25, 31, 27, 29, 28, 26}};
    static const int kRot[4][4] = {{3, 23, 17, 27}, {28, 19, 22, 7}, {29, 9, 15, 5}, {4, 13, 10, 25}};
    static const int kPerm[7] = {1, 6, 2, 3, 5, 7, 4};  // lane permutation n -> n ^ kPerm[k]
    SimdState s;
    u32 saved[32];
    std::memcpy(saved, state, sizeof saved);
    for (int i = 0; i < 8; ++i) {
        s.A[i] = state[i] ^ load_le32(blk + 4 * i);
        s.B[i] = state[8 + i] ^ load_le32(blk + 32 + 4 * i);
        s.C[i] = state[16 + i] ^ load_le32(blk + 64 + 4 * i);
        s.D[i] = state[24 + i] ^ load_le32(blk + 96 + 4 * i);
    }
    for (int r = 0; r < 4; ++r)
        for (int j = 0; j < 8; ++j) {
            const int sb = kSb[r][j];
            u32 w[8];
            for (int k = 0; k < 8; ++k) {
                if (r < 2)
                    w[k] = inner(q[16 * sb + 2 * k], q[16 * sb + 2 * k + 1], 185);
                else {
                    const int base = 16 * (sb - 8 * r) + 2 * k + (r == 3 ? 1 : 0);
                    w[k] = inner(q[base], q[base + 128], 233);
                }
            }
            const int* rot = kRot[r];
            s.step(w, j >= 4, rot[j & 3], rot[(j + 1) & 3], kPerm[(j + r) % 7]);
        }
    // feed-forward: the saved chaining value as message, IF, rotations chained from round 3
    static const int kFf[4][3] = {{4, 13, 4}, {13, 10, 5}, {10, 25, 6}, {25, 4, 0}};
    for (int k = 0; k < 4; ++k) s.step(saved + 8 * k, 0, kFf[k][0], kFf[k][1], kPerm[kFf[k][2]]);
    for (int i = 0; i < 8; ++i) {
        state[i] = s.A[i];
        state[8 + i] = s.B[i];
        state[16 + i] = s.C[i];
        state[24 + i] = s.D[i];
    }
}

void simd_compress(u32 state[32], const u8 blk[128], bool last) {
    int q[256];
    simd_expand(blk, last, q);
    simd_rounds(state, blk, q);
}

}  // namespace

Hash512 simd512(const u8* data, size_t n) {
    static const u32 kIV[32] = {
        0x0BA16B95, 0x72F999AD, 0x9FECC2AE, 0xBA3264FC, 0x5E894929, 0x8E9F30E5, 0x2F1DAA37, 0xF0F2C558,
        0xAC506643, 0xA90635A5, 0xE25B878B, 0xAAB7878F, 0x88817F7A, 0x0A02892B, 0x559A7550, 0x598F657E,
        0x7EEF60A1, 0x6B70E3E8, 0x9C1714D1, 0xB958E2A8, 0xAB02675E, 0xED1C014F, 0xCD8D65BB, 0xFDB7A257,
        0x09254899, 0xD699C7BC, 0x9019B6DC, 0x2B9022E4, 0x8FA14956, 0x21BF9BD3, 0xB94D0943, 0x6FFDDC22};
    u32 st[32];
    std::memcpy(st, kIV, sizeof st);
    const u64 bits = u64(n) * 8;
    for (; n >= 128; n -= 128, data += 128) simd_compress(st, data, false);
    u8 buf[128] = {0};
    if (n) {
        std::memcpy(buf, data, n);
        simd_compress(st, buf, false);
        std::memset(buf, 0, sizeof buf);
    }
    store_le64(buf, bits);
    if (bits == 64 * 8 || bits == 80 * 8)
        simd_rounds(st, buf, bits == 64 * 8 ? simd_final().q64 : simd_final().q80);
    else
        simd_compress(st, buf, true);
    Hash512 out;
    for (int i = 0; i < 16; ++i) store_le32(out.bytes + 4 * i, st[i]);
    return out;
}

}  // namespace nodexa
