// X16R primitives over 4-bit / bit-sliced state: JH-512, Luffa-512, Hamsi-512.
//
// Parity: sph_jh512 / sph_luffa512 / sph_hamsi512 (slots 3, 6 and 11 of HashX16R,
// src/hash.h:335-462). Written from the SHA-3 round-3 / round-2 specifications;
// round constants are generated, not stored, wherever the spec defines them
// procedurally (JH: R6 iterated from the fractional bits of sqrt(2)).
#include "x16r_prims.hpp"

#include <stdexcept>

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

// Bit-sliced E8 (the JH submission's bitslice form, derived here from the element form above):
// H is eight 128-bit words x0..x7 (16 bytes each). Element i < 128 of the grouping holds bits i of
// x0, x2, x4, x6 (its bits 3..0); element i + 128 the same bits of x1, x3, x5, x7; element-form
// pairs (A[2p], A[2p+1]) are position p of the even and the odd words. Then R8's S-box layer is
// the 4-bit S-boxes evaluated bitwise (a ten-operation circuit, the round-constant mask picking
// S1), L is eight word XORs, and P8 becomes, with the element order relabelled every
// round, a swap of the odd words' positions p <-> p ^ 2^(r mod 7); after 42 rounds the relabelling
// is the identity again. JhBitslice tracks that relabelling to place each round's constant bits
// (and the construction is checked: the pairing, the final identity and the S-box circuit against
// S0 / S1 are asserted).
// S0 / S1 of four bit planes (m0 = element bit 3 .. m3 = bit 0), the round-constant mask cc
// choosing S1: ten boolean operations per 64 elements.
inline void jh_sbox(u64& m0, u64& m1, u64& m2, u64& m3, u64 cc) {
    m3 = ~m3;
    m0 ^= ~m2 & cc;
    const u64 t0 = cc ^ (m0 & m1);
    m0 ^= m2 & m3;
    m3 ^= ~m1 & m2;
    m1 ^= m0 & m2;
    m2 ^= m0 & ~m3;
    m0 ^= m1 | m3;
    m3 ^= m1 & m2;
    m1 ^= t0 & m0;
    m2 ^= t0;
}

struct JhBitslice {
    u64 c[42][2][2];   // round, word parity (even / odd words), 128-bit mask as (bytes 0-7, 8-15) LE
    JhBitslice() {
        static const JhConstants k;
        int M[2][128];  // element index (element form, start of round r) of word parity g, position p
        for (int g = 0; g < 2; ++g)
            for (int p = 0; p < 128; ++p) M[g][p] = 2 * p + g;
        auto p8 = [](int e) {
            if (e % 4 == 2) e += 1;
            else if (e % 4 == 3) e -= 1;
            int i = e % 2 == 0 ? e / 2 : (e - 1) / 2 + 128;
            return i >= 128 ? i ^ 1 : i;
        };
        for (int r = 0; r < 42; ++r) {
            for (int g = 0; g < 2; ++g) {
                c[r][g][0] = c[r][g][1] = 0;
                for (int p = 0; p < 128; ++p) {
                    if (g == 0 && (M[0][p] % 2 != 0 || M[1][p] != M[0][p] + 1))
                        throw std::logic_error("JH bitslice: element pairing broken");
                    if (k.sel[r][M[g][p]]) c[r][g][p >> 6] |= u64(1) << (8 * ((p >> 3) & 7) + 7 - (p & 7));
                }
            }
            int n[2][128];
            const int s = 1 << (r % 7);
            for (int p = 0; p < 128; ++p) {
                n[0][p] = p8(M[0][p]);
                n[1][p ^ s] = p8(M[1][p]);
            }
            std::memcpy(M, n, sizeof M);
        }
        for (int g = 0; g < 2; ++g)
            for (int p = 0; p < 128; ++p)
                if (M[g][p] != 2 * p + g) throw std::logic_error("JH bitslice: relabelling not the identity");
        for (int cc = 0; cc < 2; ++cc)  // the bitsliced S-box circuit is S0 / S1 on every input
            for (int x = 0; x < 16; ++x) {
                u64 m0 = (x >> 3) & 1, m1 = (x >> 2) & 1, m2 = (x >> 1) & 1, m3 = x & 1;
                jh_sbox(m0, m1, m2, m3, u64(cc));
                if (int(((m0 & 1) << 3) | ((m1 & 1) << 2) | ((m2 & 1) << 1) | (m3 & 1)) != kJhS[cc][x])
                    throw std::logic_error("JH bitslice: S-box circuit");
            }
    }
};

const JhBitslice& jh_bitslice() {
    static const JhBitslice t;
    return t;
}

// Swap positions p <-> p ^ 2^k of a 128-bit word (positions: byte p / 8, bit 7 - p % 8).
inline void jh_swap(u64 w[2], int k) {
    static const u64 kMask[6] = {0x5555555555555555ULL, 0x3333333333333333ULL, 0x0F0F0F0F0F0F0F0FULL,
                                 0x00FF00FF00FF00FFULL, 0x0000FFFF0000FFFFULL, 0x00000000FFFFFFFFULL};
    if (k == 6) {
        std::swap(w[0], w[1]);
        return;
    }
    // position bits 0-2 pick the bit in the byte (7 - p % 8: flipping bit k of p flips bit k of
    // it), bits 3-5 the byte in the u64: either way p ^ 2^k is physical bit ^ 2^k
    const int sh = 1 << k;
    const u64 m = kMask[k];
    for (int h = 0; h < 2; ++h) w[h] = ((w[h] & m) << sh) | ((w[h] >> sh) & m);
}

void jh_e8(u8 H[128]) {
    const JhBitslice& B = jh_bitslice();
    u64 x[8][2];
    for (int j = 0; j < 8; ++j) {
        x[j][0] = load_le64(H + 16 * j);
        x[j][1] = load_le64(H + 16 * j + 8);
    }
    for (int r = 0; r < 42; ++r) {
        for (int g = 0; g < 2; ++g)
            for (int h = 0; h < 2; ++h) {
                jh_sbox(x[g][h], x[2 + g][h], x[4 + g][h], x[6 + g][h], B.c[r][g][h]);
            }
        for (int h = 0; h < 2; ++h) {  // L: odd words ^= mul2(even words), then even ^= mul2(odd)
            x[1][h] ^= x[2][h];
            x[3][h] ^= x[4][h];
            x[5][h] ^= x[6][h] ^ x[0][h];
            x[7][h] ^= x[0][h];
            x[0][h] ^= x[3][h];
            x[2][h] ^= x[5][h];
            x[4][h] ^= x[7][h] ^ x[1][h];
            x[6][h] ^= x[1][h];
        }
        for (int j = 1; j < 8; j += 2) jh_swap(x[j], r % 7);
    }
    for (int j = 0; j < 8; ++j) {
        store_le64(H + 16 * j, x[j][0]);
        store_le64(H + 16 * j + 8, x[j][1]);
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

// ================================================================ Luffa-512 (w = 5)
// Five 256-bit lanes V_j (8 x u32), message injection MI5 over GF(2^8)^32 (x2 = the
// M2 word shift with taps 0, 1, 3, 4), tweak (lane j words 4..7 rotated by j), then
// 8 steps per lane of SubCrumb / MixWord / AddConstant. Blank rounds squeeze 2 x 256.
namespace {

// Starting values and step constants of Luffa v2 (spec tables, big-endian hex).
const char* const kLuffaIV =
    "6d251e6944b051e04eaa6fb4dbf784656e29201190152df4ee058139def610bb"
    "c3b44b95d9d2f25670eee9a0de099fa35d9b05578fc944b3cf1ccf0e746cd581"
    "f7efc89d5dba578104016ce5ad659c050306194f666d183624aa230a8b264ae7"
    "858075d536d79ccee571f7d7204b1f6735870c6a57e9e92314bcb8087cde72ce"
    "6c68e9be5ec41e22c825b7c7affb4363f5df39990fc688f1b07224cc03e86cea";
const char* const kLuffaRC[5][2] = {
    {"303994a6c0e652996cc33a12dc56983e1e00108f7800423d8f5b788296e1db12",
     "e0337818441ba90d7f34d4429389217fe5a8bce65274baf426889ba79a226e9d"},
    {"b6de10ed70f47aae0707a3d41c1e8f51707a3d45aeb28562baca158940a46f3e",
     "01685f3d05a17cf4bd09cacaf4272b28144ae5ccfaa7ae2b2e48f1c1b923c704"},
    {"fc20d9d234552e257ad8818f8438764abb6de032edb780c8d9847356a2c78434",
     "e25e72c1e623bb725c58a4a41e38e2e778e38b9d2758671936eda57f703aace7"},
    {"b213afa5c84ebe954e608a2256d858fe343b138fd0ec4e3d2ceb4882b3ad2208",
     "e028c9bf44756f917e8fce32956548befe191be23cb226e55944a28ea1c4c355"},
    {"f0d2e9e3ac11d7fa1bcb66f26f2d9bc9786026498edae9523b6ba548edae9520",
     "5090d5772d1925abb46496acd1925ab029131ab60fc053c33f014f0cfc053c31"}};

void hex_words(const char* h, u32* out, int n) {
    for (int i = 0; i < n; ++i) {
        u32 v = 0;
        for (int k = 0; k < 8; ++k) {
            const char c = h[8 * i + k];
            v = (v << 4) | u32(c <= '9' ? c - '0' : c - 'a' + 10);
        }
        out[i] = v;
    }
}

struct LuffaConst {
    u32 iv[5][8], rc[5][2][8];
    LuffaConst() {
        hex_words(kLuffaIV, &iv[0][0], 40);
        for (int j = 0; j < 5; ++j)
            for (int k = 0; k < 2; ++k) hex_words(kLuffaRC[j][k], rc[j][k], 8);
    }
};

using Lane = u32[8];

void luffa_x2(Lane& d, const Lane& s) {
    const u32 t = s[7];
    u32 r[8] = {t, s[0] ^ t, s[1], s[2] ^ t, s[3] ^ t, s[4], s[5], s[6]};
    std::memcpy(d, r, sizeof r);
}

void luffa_xor(Lane& d, const Lane& a, const Lane& b) {
    for (int i = 0; i < 8; ++i) d[i] = a[i] ^ b[i];
}

void sub_crumb(u32& a0, u32& a1, u32& a2, u32& a3) {
    u32 t = a0;
    a0 |= a1; a2 ^= a3; a1 = ~a1; a0 ^= a3; a3 &= t; a1 ^= a3; a3 ^= a2; a2 &= a0;
    a0 = ~a0; a2 ^= a1; a1 |= a3; t ^= a1; a3 ^= a2; a2 &= a1; a1 ^= a0; a0 = t;
}

void mix_word(u32& u, u32& v) {
    v ^= u;
    u = rotl32(u, 2) ^ v;
    v = rotl32(v, 14) ^ u;
    u = rotl32(u, 10) ^ v;
    v = rotl32(v, 1);
}

void luffa_round(Lane V[5], const u8 blk[32], const LuffaConst& k) {
    Lane M, a, b;
    for (int i = 0; i < 8; ++i) M[i] = load_be32(blk + 4 * i);
    // MI5
    luffa_xor(a, V[0], V[1]);
    luffa_xor(b, V[2], V[3]);
    luffa_xor(a, a, b);
    luffa_xor(a, a, V[4]);
    luffa_x2(a, a);
    for (int j = 0; j < 5; ++j) luffa_xor(V[j], V[j], a);
    luffa_x2(b, V[0]);
    luffa_xor(b, b, V[1]);
    for (int j = 1; j < 4; ++j) { luffa_x2(V[j], V[j]); luffa_xor(V[j], V[j], V[j + 1]); }
    luffa_x2(V[4], V[4]);
    luffa_xor(V[4], V[4], V[0]);
    luffa_x2(V[0], b);
    luffa_xor(V[0], V[0], V[4]);
    for (int j = 4; j > 1; --j) { luffa_x2(V[j], V[j]); luffa_xor(V[j], V[j], V[j - 1]); }
    luffa_x2(V[1], V[1]);
    luffa_xor(V[1], V[1], b);
    for (int j = 0; j < 5; ++j) {
        if (j) luffa_x2(M, M);
        luffa_xor(V[j], V[j], M);
    }
    // tweak + Q_j
    for (int j = 0; j < 5; ++j) {
        u32* x = V[j];
        for (int i = 4; i < 8; ++i) x[i] = rotl32(x[i], j);
        for (int r = 0; r < 8; ++r) {
            sub_crumb(x[0], x[1], x[2], x[3]);
            sub_crumb(x[5], x[6], x[7], x[4]);
            for (int i = 0; i < 4; ++i) mix_word(x[i], x[i + 4]);
            x[0] ^= k.rc[j][0][r];
            x[4] ^= k.rc[j][1][r];
        }
    }
}

}  // namespace

Hash512 luffa512(const u8* data, size_t n) {
    static const LuffaConst k;
    Lane V[5];
    std::memcpy(V, k.iv, sizeof V);
    for (; n >= 32; n -= 32, data += 32) luffa_round(V, data, k);
    u8 buf[32] = {0};
    std::memcpy(buf, data, n);
    buf[n] = 0x80;
    luffa_round(V, buf, k);
    Hash512 out;
    const u8 zero[32] = {0};
    for (int half = 0; half < 2; ++half) {
        luffa_round(V, zero, k);
        for (int i = 0; i < 8; ++i)
            store_be32(out.bytes + 32 * half + 4 * i, V[0][i] ^ V[1][i] ^ V[2][i] ^ V[3][i] ^ V[4][i]);
    }
    return out;
}

// ================================================================ Hamsi-512
// 64-bit message blocks expanded by the spec's linear code to 512 bits (one row of
// kHamsiExpand per message bit, bits of each byte least-significant first),
// concatenated with the 512-bit chaining value into a 32-word state; 6 rounds
// (12 with the final-block constants) of constant add, the 4-bit S-box bitsliced
// over 4 words, and the Serpent-style diffusion L; truncation + feed-forward.
namespace {

const char* const kHamsiExpand[64] = {
    "ef0b02703afd00005dae0000694900009b0f3c064405b5f966140a51924f5d0ac96b0030e72500002f840000264f000008695bf96dfcf137509f69849e69af68",
    "c96b0030e72500002f840000264f000008695bf96dfcf137509f69849e69af6826600240ddd80000722a00004f060000936667ff29f944ce368b63d50c26f262",
    "145a3c00b9e9000061270000f1610000ce613d6cb0493d7847a96720e18e24c523671400c8b90000f4c70000fb75000073cd2465f8a6a54902c40a3fdc24e61f",
    "23671400c8b90000f4c70000fb75000073cd2465f8a6a54902c40a3fdc24e61f373d28007150000095e000000a140000bdac190948ef9831456d6d1f3daac2da",
    "54285c00eaed0000c5d60000a1c50000b3a2677094a5c4e16bb0419d551b37829cbb1800b0d3000092510000ed930000593a4345e114d5f4430633da78cace29",
    "9cbb1800b0d3000092510000ed930000593a4345e114d5f4430633da78cace29c89344005a3e0000578700004c560000ea98243575b1111528b672472dd1f9ab",
    "29449c0064e70000f24b0000c2f300000ede4e8f56c23745f3e042598d0d9ec4466d0c0008620000dd5d0000badd00006a927942441f2b93218ace6fbf2c0be2",
    "466d0c0008620000dd5d0000badd00006a927942441f2b93218ace6fbf2c0be26f2990006c8500002f160000782e0000644c37cd12dd1cd6d26a8c3632219526",
    "f68000053443c000240700008f3d000021373bfb0ab8d5aecdc58b19d795ba31a67f00017137800019fc000096db00003a8b6dfdebcaaef32c6d478fac8e6c88",
    "a67f00017137800019fc000096db00003a8b6dfdebcaaef32c6d478fac8e6c8850ff0004457440003dfb000019e600001bbc5606e1727b5de1a8cc967b1bd6b9",
    "f7750009cf3cc000c3d6000004920000029519a9f8e836ba7a87f14e9e16981ad46a00008dc8c000a5af00004a290000fc4e427ac9b4866c98369604f746c320",
    "d46a00008dc8c000a5af00004a290000fc4e427ac9b4866c98369604f746c320231f000942f40000667900004ebb0000fedb5bd3315cb0d6e2b1674a69505b3a",
    "774400f0f15a0000f5b200003414000089377e8c5a8bec250bc3cd1ecf3775cbf46c00509618000014a50000031f000042947eb866bf7e199ca470d28a341574",
    "f46c00509618000014a50000031f000042947eb866bf7e199ca470d28a341574832800a067420000e1170000370b0000cba300343c34923c9767bdcc450360bf",
    "e88701709d72000012db0000d4220000f2886b27a921e5434ef8b518618813b1b43700600c4c000056c200005cae000094541f3f3b3ef8251b365f3df3d45758",
    "b43700600c4c000056c200005cae000094541f3f3b3ef8251b365f3df3d457585cb00110913e000044190000888c000066dc7418921f1d6655ceea25925c44e9",
    "0c72000049e50f00427900005cea000033aa301a1582251495a34b7bb44b0090fe220000a758050025d10000f7600000893178da1fd4f8604ed0a315a123ff9f",
    "fe220000a758050025d10000f7600000893178da1fd4f8604ed0a315a123ff9ff2500000eebd0a0067a80000ab8a0000ba9b48c00a56dd74db73e86e1568ff0f",
    "45180000a5b51700f96a00003b4800001ecc142c231395d616bca6b0df33f4dfb83d000016710600379a0000f5b10000228161acae48f14566241616c5c1eb3e",
    "b83d000016710600379a0000f5b10000228161acae48f14566241616c5c1eb3efd250000b3c41100cef00000cef900003c4d75808d5b64937098b0a61af21fe1",
    "75a40000c28b270094a4000090f50000fb7857e049ce0bae1767c483aedf667ed16600001bbc03009eec0000f694000003024527cf70fcf2b4431b17857f3c2b",
    "d16600001bbc03009eec0000f694000003024527cf70fcf2b4431b17857f3c2ba4c20000d93724000a48000066610000f87a12c786bef75ca324df942ba05a55",
    "75c900030e10c000d1200000baea00008bc42f3e8758b757bb28761d00b72e2beecf00016f564000f33e0000a79e0000bdb57219b711ebc54a3b40bafeabf254",
    "eecf00016f564000f33e0000a79e0000bdb57219b711ebc54a3b40bafeabf2549b06000261468000221e00001d74000036715d2730495c92f11336a7fe1cdc7f",
    "867900003f390002e19ae000985600009565670e4e88c8ead3dd4944161ddab930b70000e5d00000f4f4600042c4000063b83d6a78ba946021afa1eab0a51834",
    "30b70000e5d00000f4f4600042c4000063b83d6a78ba946021afa1eab0a51834b6ce0000dae90002156e8000da920000f6dd5a6436325c8af272e8aea6b8c28d",
    "1419000023ca003c50df000044b600001b6c67b03cf3ac7561e610b0dbcadb80e34300003a4e0014f2c60000aa4e0000db1e42a6256bbe15123db1563a4e99d7",
    "e34300003a4e0014f2c60000aa4e0000db1e42a6256bbe15123db1563a4e99d7f75a000019840028a2190000eef80000c07225161998126073dba1e6e1844257",
    "545000000671005c25ae00006a1e00002ea54edf664e8512bfba18c37e715d17bc8d0000fc3b001819830000d10b0000ae1878c442a698560012da372c3b504e",
    "bc8d0000fc3b001819830000d10b0000ae1878c442a698560012da372c3b504ee8dd0000fa4a00443c2d0000bb15000080bd361b24e81d44bfa8c2f4524a0d59",
    "69510000d4e1009cc3230000ac2f0000e4950baecea415dc87ec287cbce1a3cec6730000af8d000ca4c10000218d0000231115877913512f1d28ac88378dd173",
    "c6730000af8d000ca4c10000218d0000231115877913512f1d28ac88378dd173af2200007b6c009067e200008da20000c7841e29b7b744f39ac484f48b6c72bd",
    "cc140000a56300005ab907803b5000004bd013ff879b3418694348c1ca5a87fe819e0000ec5700006632028095f300005da9280248f43cbce65aa22d8e67b7fa",
    "819e0000ec5700006632028095f300005da9280248f43cbce65aa22d8e67b7fa4d8a0000493400003c8b0500aea3000016793bfdcf6f08a48f19eaec443d3004",
    "7823000012fc0000a93a0b8090a50000713e28797ee98924f08ca062636f8bab02af0000b7280000ba1c030056980000ba8d45d38048c667a95c149af4f6ea7b",
    "02af0000b7280000ba1c030056980000ba8d45d38048c667a95c149af4f6ea7b7a8c0000a5d4000013260880c63d0000cbb36daafea14f4359d0b4f8979961d0",
    "ac4800001ba6000045fb1380034300005a85316a1fb250b6fe72c7fe91e478f61e4e0000decf00006df8018077240000ec47079ef4a0694ecda3181298aa496e",
    "1e4e0000decf00006df8018077240000ec47079ef4a0694ecda3181298aa496eb2060000c56900002803120074670000b6c236f4eb1239f833d1dfec094e3198",
    "aec300009c4f000179d1e0002c15000045cc75b36650b736ab92f78fa312567bdb2500000929000049aac00081e10000cafe6b594279343143566b76e86cba2e",
    "db2500000929000049aac00081e10000cafe6b594279343143566b76e86cba2e75e6000095660001307b2000adf400008f321eea24298307e8c49cf94b7eec55",
    "58430000807e000078330001c66b3800e7375cdc79ad3fddac73fe6f3a4479b11d5a00002b720000488d0000af61180025cb2ec5c879bfd081a204291e7536a6",
    "1d5a00002b720000488d0000af61180025cb2ec5c879bfd081a204291e7536a645190000ab0c000030be0001690a2000c2fc7219b1d4800d2dd1fa4624314f17",
    "a53b0000142600004e30001e7cae00008f9e0dd578dfaa3df73168d80b1b494607ed0000b25000008774000a970d0000437223ae48c76ea4f47862229075b1ce",
    "07ed0000b25000008774000a970d0000437223ae48c76ea4f47862229075b1cea2d60000a6760000c9440014eba30000ccec2e7b3018c49903490afa9b6ef888",
    "889800001f9400007fcf002efb4e0000f158079a61ae9167a895706ce61074940bc20000db6300007e88000c1586000091fd48f37581bb43f460449ed8b61463",
    "0bc20000db6300007e88000c1586000091fd48f37581bb43f460449ed8b61463835a0000c4f7000001470022eec8000060a54f69142f2a245cf534f23ea660f7",
    "52500000295400006a61004ef0ff00009a317eec452341cecf568fe55303130f538d0000a9fc00009ef7000656ff00000ae4004e92c5cdf9a94440187f975691",
    "538d0000a9fc00009ef7000656ff00000ae4004e92c5cdf9a94440187f97569101dd000080a80000f4960048a600000090d57ea2d7e68c376612cffd2c94459e",
    "e62800004c4b0000a8550000d3d002e0d86130b898a7b0da289506b4d75a4897f0c500005923000045820000e18d00c03b6d0631c2ed5699cbe0fe1c56a7b19f",
    "f0c500005923000045820000e18d00c03b6d0631c2ed5699cbe0fe1c56a7b19f16ed000015680000edd70000325d0220e30c36895a4ae643e375f8a881fdf908",
    "b431000077330000b15d00007fd004e078a26138d116c35dd256d4894e6f74dee3060000bdc1000087130000bff200602eba0a1a8db5375173c5ab065bd61539",
    "e3060000bdc1000087130000bff200602eba0a1a8db5375173c5ab065bd6153957370000caf20000364e0000c022048056186b225ca3f40ca1937f8f15b961e7",
    "02f20000a2810000873f0000e36c78001e1d74ef073d2bd6c4c232377f32259ebadd000013ad0000b7e70000f7282800df45144d361ac33aea5a8d142a2c18f0",
    "badd000013ad0000b7e70000f7282800df45144d361ac33aea5a8d142a2c18f0b82f0000b12c000030d8000014445000c15860a23127e8ec2e98bf23551e3d6e",
    "1e6c0000c44200008a2e0000bcb6b8002c4413b68bfdd3da6a0c1bc8b99dc2eb925600001eda0000ea510000e8b13000a93556a5ebfb6199b15c225433c5244f",
    "925600001eda0000ea510000e8b13000a93556a5ebfb6199b15c225433c5244f8c3a0000da980000607f000054078800857145136006b243db50399c8a58e6a4",
    "033d000008b30000f33a00003ac2000751298a506b6e661f0ea5cfe3e6da7ffea8da000096be00005c1d000007da00027d6695831f98708abb668808da878000",
    "a8da000096be00005c1d000007da00027d6695831f98708abb668808da878000abe700009e0d0000af2700003d1800052c4f1fd374f61695b5c347eb3c5dfffe",
    "01930000e7820000edfb0000cf0c000b8dd08d58bca3b42e063661e1536f9e7b92280000dc85000057fa000056dc0003bae923165aefa30c90cef7527b1675d7",
    "92280000dc85000057fa000056dc0003bae923165aefa30c90cef7527b1675d793bb00003b070000ba01000099d000083739ae4ee64c172296f896b32879ebac",
    "5fa800005603000043ae000064f30013257e86bf1311944e541e95bf8ea4db69004400007f480000da7c00002a2300013badc9cca9b69c87030a9e60be0a679e",
    "004400007f480000da7c00002a2300013badc9cca9b69c87030a9e60be0a679e5fec0000294b000099d200004ed000121ed34f73baa708c957140bdf30aebcf7",
    "ee930000d607000092c100002b9801e09451287c3b6cfb5745312374201f6a647b28000057420000a9e50000634300a09edb442f6d9995bb27f83b03c7ff60f0",
    "7b28000057420000a9e50000634300a09edb442f6d9995bb27f83b03c7ff60f095bb0000814500003b24000048db01400a8a6c5356f56eec62c91877e7e00a94",
};
const char* const kHamsiAlphaN = "ff00f0f0ccccaaaaf0f0ccccff00aaaaccccaaaaf0f0ff00aaaaccccf0f0ff00f0f0ccccaaaaff00ccccff00aaaaf0f0aaaaf0f0ff00ccccccccf0f0ff00aaaaccccaaaaff00f0f0ff00aaaaf0f0ccccf0f0ff00ccccaaaaf0f0ff00aaaaccccaaaaff00f0f0ccccaaaaf0f0ccccff00ff00ccccaaaaf0f0ff00aaaaccccf0f0";
const char* const kHamsiAlphaF = "caf9639c0ff0f9c0639c0ff0caf9f9c00ff0f9c0639ccaf9f9c00ff0639ccaf9639c0ff0f9c0caf90ff0caf9f9c0639cf9c0639ccaf90ff00ff0639ccaf9f9c00ff0f9c0caf9639ccaf9f9c0639c0ff0639ccaf90ff0f9c0639ccaf9f9c00ff0f9c0caf9639c0ff0f9c0639c0ff0caf9caf90ff0f9c0639ccaf9f9c00ff0639c";

struct HamsiConst {
    u32 T[64][16], an[32], af[32], iv[16];
    HamsiConst() {
        for (int i = 0; i < 64; ++i) hex_words(kHamsiExpand[i], T[i], 16);
        hex_words(kHamsiAlphaN, an, 32);
        hex_words(kHamsiAlphaF, af, 32);
        // IV: the designers' address as 16 big-endian words
        static const char addr[] = "steelpark Arenberg 10, bus 2446, B-3001 Leuven-Heverlee, Belgium";
        for (int i = 0; i < 16; ++i) iv[i] = load_be32(reinterpret_cast<const u8*>(addr) + 4 * i);
    }
};

void hamsi_sbox(u32& a, u32& b, u32& c, u32& d) {
    u32 t = a;
    a &= c; a ^= d; c ^= b; c ^= a; d |= t; d ^= b; t ^= c; b = d; d |= t; d ^= a;
    a &= b; t ^= a; b ^= d; b ^= t; a = c; c = b; b = d; d = ~t;
}

void hamsi_L(u32& a, u32& b, u32& c, u32& d) {
    a = rotl32(a, 13);
    c = rotl32(c, 3);
    b ^= a ^ c;
    d ^= c ^ (a << 3);
    b = rotl32(b, 1);
    d = rotl32(d, 7);
    a ^= b ^ d;
    c ^= d ^ (b << 7);
    a = rotl32(a, 5);
    c = rotl32(c, 22);
}

void hamsi_block(u32 h[16], const u8 blk[8], bool final, const HamsiConst& k) {
    u32 m[16] = {0};
    for (int u = 0; u < 8; ++u)
        for (int v = 0; v < 8; ++v)
            if ((blk[u] >> v) & 1)
                for (int w = 0; w < 16; ++w) m[w] ^= k.T[8 * u + v][w];
    // state layout: (m0 m1 c0 c1 m2 m3 c2 c3 c4 c5 m4 m5 c6 c7 m6 m7 | same for +8)
    static const int kSlot[32] = {0, 1, 16, 17, 2, 3, 18, 19, 20, 21, 4, 5, 22, 23, 6, 7,
                                  8, 9, 24, 25, 10, 11, 26, 27, 28, 29, 12, 13, 30, 31, 14, 15};
    u32 mc[32];
    for (int i = 0; i < 16; ++i) { mc[i] = m[i]; mc[16 + i] = h[i]; }
    u32 s[32];
    for (int i = 0; i < 32; ++i) s[i] = mc[kSlot[i]];
    const u32* alpha = final ? k.af : k.an;
    const int rounds = final ? 12 : 6;
    for (int r = 0; r < rounds; ++r) {
        for (int i = 0; i < 32; ++i) s[i] ^= alpha[i];
        s[1] ^= u32(r);
        for (int i = 0; i < 8; ++i) hamsi_sbox(s[i], s[i + 8], s[i + 16], s[i + 24]);
        for (int i = 0; i < 8; ++i) hamsi_L(s[i], s[8 + ((i + 1) & 7)], s[16 + ((i + 2) & 7)], s[24 + ((i + 3) & 7)]);
        hamsi_L(s[0x00], s[0x02], s[0x05], s[0x07]);
        hamsi_L(s[0x10], s[0x13], s[0x15], s[0x16]);
        hamsi_L(s[0x09], s[0x0B], s[0x0C], s[0x0E]);
        hamsi_L(s[0x19], s[0x1A], s[0x1C], s[0x1F]);
    }
    for (int i = 0; i < 8; ++i) {
        h[i] ^= s[i];
        h[8 + i] ^= s[16 + i];
    }
}

}  // namespace

Hash512 hamsi512(const u8* data, size_t n) {
    static const HamsiConst k;
    u32 h[16];
    std::memcpy(h, k.iv, sizeof h);
    const u64 bits = u64(n) * 8;
    for (; n >= 8; n -= 8, data += 8) hamsi_block(h, data, false, k);
    u8 last[8] = {0}, len[8];
    std::memcpy(last, data, n);
    last[n] = 0x80;
    hamsi_block(h, last, false, k);
    store_be64(len, bits);
    hamsi_block(h, len, true, k);
    Hash512 out;
    for (int i = 0; i < 16; ++i) store_be32(out.bytes + 4 * i, h[i]);
    return out;
}


}  // namespace nodexa
