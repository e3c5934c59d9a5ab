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

// The same round on four little-endian column words through the usual four 256 x u32 tables:
// T[k][x] is the MixColumns image of S[x] entering at row k (T[0][x] bytes 2S, S, S, 3S).
struct AesT {
    u32 T[4][256];
    AesT() {
        const u8* S = aes_sbox();
        for (int x = 0; x < 256; ++x) {
            const u8 s = S[x], s2 = xtime(s), s3 = u8(s2 ^ s);
            const u32 v = u32(s2) | (u32(s) << 8) | (u32(s) << 16) | (u32(s3) << 24);
            for (int k = 0; k < 4; ++k) T[k][x] = k ? rotl32(v, 8 * k) : v;
        }
    }
};

const AesT& aes_t() {
    static const AesT t;
    return t;
}

inline void aes_round_w(u32 x[4], const u32* key, const AesT& A) {
    const u32 y0 = A.T[0][x[0] & 0xFF] ^ A.T[1][(x[1] >> 8) & 0xFF] ^ A.T[2][(x[2] >> 16) & 0xFF] ^ A.T[3][x[3] >> 24];
    const u32 y1 = A.T[0][x[1] & 0xFF] ^ A.T[1][(x[2] >> 8) & 0xFF] ^ A.T[2][(x[3] >> 16) & 0xFF] ^ A.T[3][x[0] >> 24];
    const u32 y2 = A.T[0][x[2] & 0xFF] ^ A.T[1][(x[3] >> 8) & 0xFF] ^ A.T[2][(x[0] >> 16) & 0xFF] ^ A.T[3][x[1] >> 24];
    const u32 y3 = A.T[0][x[3] & 0xFF] ^ A.T[1][(x[0] >> 8) & 0xFF] ^ A.T[2][(x[1] >> 16) & 0xFF] ^ A.T[3][x[2] >> 24];
    x[0] = y0 ^ (key ? key[0] : 0);
    x[1] = y1 ^ (key ? key[1] : 0);
    x[2] = y2 ^ (key ? key[2] : 0);
    x[3] = y3 ^ (key ? key[3] : 0);
}

// xtime on four packed bytes
inline u32 xtime4(u32 v) { return ((v & 0x7F7F7F7Fu) << 1) ^ (((v >> 7) & 0x01010101u) * 0x1Bu); }

}  // namespace

// ================================================================ Groestl-512
// 16 columns of 8 bytes (u64, row i in byte i), P1024 / Q1024 with 14 rounds each. SubBytes,
// ShiftBytes and MixBytes fold into eight 256 x u64 tables: T[k][x] is the column that byte x
// in row k contributes after the S-box and the circulant circ(2,2,3,4,5,3,5,7), so a round is 8
// lookups per output column (the tables are derived here from the S-box and GF(2^8)).
namespace {

struct GroestlTables {
    u64 T[8][256];
    GroestlTables() {
        static const u8 kMix[8] = {2, 2, 3, 4, 5, 3, 5, 7};
        const u8* S = aes_sbox();
        for (int k = 0; k < 8; ++k)
            for (int x = 0; x < 256; ++x) {
                u64 v = 0;
                for (int i = 0; i < 8; ++i) v |= u64(gmul(S[x], kMix[(k - i) & 7])) << (8 * i);
                T[k][x] = v;
            }
    }
};

const GroestlTables& groestl_tables() {
    static const GroestlTables t;
    return t;
}

void groestl_perm(u64 st[16], bool q) {
    static const int kShiftP[8] = {0, 1, 2, 3, 4, 5, 6, 11};
    static const int kShiftQ[8] = {1, 3, 5, 11, 0, 2, 4, 6};
    const GroestlTables& G = groestl_tables();
    const int* sh = q ? kShiftQ : kShiftP;
    u64 t[16];
    for (int r = 0; r < 14; ++r) {
        for (int j = 0; j < 16; ++j)  // AddRoundConstant
            st[j] ^= q ? ~(u64((j << 4) ^ r) << 56) : u64((j << 4) ^ r);
        for (int j = 0; j < 16; ++j) {
            u64 v = 0;
            for (int k = 0; k < 8; ++k) v ^= G.T[k][u8(st[(j + sh[k]) & 15] >> (8 * k))];
            t[j] = v;
        }
        std::memcpy(st, t, sizeof t);
    }
}

void groestl_compress(u64 h[16], const u8 m[128]) {
    u64 p[16], q[16];
    for (int j = 0; j < 16; ++j) {
        q[j] = load_le64(m + 8 * j);
        p[j] = h[j] ^ q[j];
    }
    groestl_perm(p, false);
    groestl_perm(q, true);
    for (int j = 0; j < 16; ++j) h[j] ^= p[j] ^ q[j];
}

}  // namespace

Hash512 groestl512(const u8* data, size_t n) {
    u64 h[16] = {0};
    h[15] = u64(0x02) << 48;  // output size 512, 64-bit big-endian at the end of the IV (byte 126)
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
    u64 x[16];
    std::memcpy(x, h, sizeof x);
    groestl_perm(x, false);
    Hash512 out;
    for (int j = 0; j < 8; ++j) store_le64(out.bytes + 8 * j, x[8 + j] ^ h[8 + j]);
    return out;
}

// ================================================================ ECHO-512
// 16 x 128-bit words; 1024-bit chaining value, 1024-bit message block, 10 rounds.
namespace {

// 16 words of 128 bits as 4 little-endian column words each; BIG.SubWords is two word rounds,
// BIG.MixColumns the AES MixColumns applied bytewise across four words (packed four bytes at once).
void echo_compress(u32 v[8][4], const u8 m[128], u64 counter_bits) {
    const AesT& A = aes_t();
    u32 w[16][4];
    for (int i = 0; i < 8; ++i)
        for (int c = 0; c < 4; ++c) w[i][c] = v[i][c];
    for (int i = 0; i < 8; ++i)
        for (int c = 0; c < 4; ++c) w[8 + i][c] = load_le32(m + 16 * i + 4 * c);
    u64 k = counter_bits;
    for (int r = 0; r < 10; ++r) {
        for (int i = 0; i < 16; ++i) {
            const u32 key[4] = {u32(k), u32(k >> 32), 0, 0};
            ++k;
            aes_round_w(w[i], key, A);
            aes_round_w(w[i], nullptr, A);
        }
        u32 t[16][4];
        for (int j = 0; j < 4; ++j)
            for (int i = 0; i < 4; ++i) std::memcpy(t[4 * j + i], w[4 * ((j + i) & 3) + i], 16);
        for (int j = 0; j < 4; ++j)
            for (int c = 0; c < 4; ++c) {
                const u32 a0 = t[4 * j][c], a1 = t[4 * j + 1][c], a2 = t[4 * j + 2][c], a3 = t[4 * j + 3][c];
                const u32 x0 = xtime4(a0), x1 = xtime4(a1), x2 = xtime4(a2), x3 = xtime4(a3);
                w[4 * j + 0][c] = x0 ^ x1 ^ a1 ^ a2 ^ a3;
                w[4 * j + 1][c] = a0 ^ x1 ^ x2 ^ a2 ^ a3;
                w[4 * j + 2][c] = a0 ^ a1 ^ x2 ^ x3 ^ a3;
                w[4 * j + 3][c] = x0 ^ a0 ^ a1 ^ a2 ^ x3;
            }
    }
    for (int i = 0; i < 8; ++i)
        for (int c = 0; c < 4; ++c) v[i][c] ^= load_le32(m + 16 * i + 4 * c) ^ w[i][c] ^ w[8 + i][c];
}

}  // namespace

Hash512 echo512(const u8* data, size_t n) {
    u32 v[8][4] = {{0}};
    for (int i = 0; i < 8; ++i) v[i][0] = 0x0200;  // 512, 128-bit little-endian
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
    for (int i = 0; i < 4; ++i)
        for (int c = 0; c < 4; ++c) store_le32(out.bytes + 16 * i + 4 * c, v[i][c]);
    return out;
}

// ================================================================ SHAvite-3-512
// HAIFA compression C512: 512-bit chaining value as four 128-bit blocks, 1024-bit
// message expanded into 448 round-key words (AES rounds + linear steps, the
// 128-bit bit counter injected at four fixed positions), 14 Feistel-like rounds
// of four keyless AES rounds per branch.
namespace {

u32 le_word(const u8* p) { return load_le32(p); }

void aes_words(u32 x[4]) { aes_round_w(x, nullptr, aes_t()); }  // one keyless AES round

void shavite_c512(u32 h[16], const u8 msg[128], const u32 cnt[4]) {
    u32 rk[448];
    for (int i = 0; i < 32; ++i) rk[i] = le_word(msg + 4 * i);
    // counter words xored into the expansion, with the fourth complemented
    auto inject = [&](int u, int a, int b, int c, int d) {
        rk[u] ^= cnt[a]; rk[u + 1] ^= cnt[b]; rk[u + 2] ^= cnt[c]; rk[u + 3] ^= ~cnt[d];
    };
    int u = 32;
    for (;;) {
        for (int s = 0; s < 8; ++s) {  // nonlinear expansion: AES of the rotated 4 words 32 back
            u32 x[4] = {rk[u - 31], rk[u - 30], rk[u - 29], rk[u - 32]};
            aes_words(x);
            for (int k = 0; k < 4; ++k) rk[u + k] = x[k] ^ rk[u - 4 + k];
            if (u == 32) inject(32, 0, 1, 2, 3);
            else if (u == 164) inject(164, 3, 2, 1, 0);
            else if (u == 316) inject(316, 2, 3, 0, 1);
            else if (u == 440) inject(440, 1, 0, 3, 2);
            u += 4;
        }
        if (u == 448) break;
        for (int s = 0; s < 8; ++s, u += 4)  // linear expansion
            for (int k = 0; k < 4; ++k) rk[u + k] = rk[u - 32 + k] ^ rk[u - 7 + k];
    }
    u32 P[4][4];
    for (int b = 0; b < 4; ++b)
        for (int k = 0; k < 4; ++k) P[b][k] = h[4 * b + k];
    int r_idx = 0;
    auto F = [&](u32 (&L)[4], const u32 (&R)[4]) {
        u32 x[4];
        for (int k = 0; k < 4; ++k) x[k] = R[k] ^ rk[r_idx++];
        aes_words(x);
        for (int j = 0; j < 3; ++j) {
            for (int k = 0; k < 4; ++k) x[k] ^= rk[r_idx++];
            aes_words(x);
        }
        for (int k = 0; k < 4; ++k) L[k] ^= x[k];
    };
    for (int r = 0; r < 14; ++r) {
        F(P[0], P[1]);
        F(P[2], P[3]);
        u32 t[4];
        std::memcpy(t, P[3], sizeof t);
        std::memcpy(P[3], P[2], sizeof t);
        std::memcpy(P[2], P[1], sizeof t);
        std::memcpy(P[1], P[0], sizeof t);
        std::memcpy(P[0], t, sizeof t);
    }
    for (int b = 0; b < 4; ++b)
        for (int k = 0; k < 4; ++k) h[4 * b + k] ^= P[b][k];
}

}  // namespace

Hash512 shavite512(const u8* data, size_t n) {
    static const u32 kIV[16] = {0x72FCCDD8, 0x79CA4727, 0x128A077B, 0x40D55AEC, 0xD1901A06, 0x430AE307,
                                0xB29F5CD1, 0xDF07FBFC, 0x8E45D73D, 0x681AB538, 0xBDE86578, 0xDD577E47,
                                0xE275EADE, 0x502D9FCD, 0xB9357178, 0x022A4B9A};
    u32 h[16];
    std::memcpy(h, kIV, sizeof h);
    const u64 bits = u64(n) * 8;
    u64 done = 0;
    for (; n >= 128; n -= 128, data += 128) {
        done += 1024;
        const u32 cnt[4] = {u32(done), u32(done >> 32), 0, 0};
        shavite_c512(h, data, cnt);
    }
    // 0x80, zeros, 128-bit bit count (LE) at 110, digest size 512 (16-bit LE) at 126
    u8 buf[128] = {0};
    std::memcpy(buf, data, n);
    const u32 total[4] = {u32(bits), u32(bits >> 32), 0, 0};
    const u32 zero[4] = {0, 0, 0, 0};
    const u32* last_cnt = total;
    if (n == 0) {
        buf[0] = 0x80;
        last_cnt = zero;  // a block with no message bits is compressed with counter 0
    } else if (n < 110) {
        buf[n] = 0x80;
    } else {
        buf[n] = 0x80;
        shavite_c512(h, buf, total);
        std::memset(buf, 0, 110);
        last_cnt = zero;
    }
    for (int i = 0; i < 4; ++i) store_le32(buf + 110 + 4 * i, total[i]);
    buf[126] = 0x00;
    buf[127] = 0x02;
    shavite_c512(h, buf, last_cnt);
    Hash512 out;
    for (int i = 0; i < 16; ++i) store_le32(out.bytes + 4 * i, h[i]);
    return out;
}

// ================================================================ Fugue-512
// 36-column state (u32 per column, row 0 in the most significant byte). Each input
// word: TIX, then four sub-rounds of ROR3 / CMIX / SMIX; SMIX = AES S-box on the
// 4x4 byte block followed by the Super-Mix matrix, evaluated through the
// column tables (S, S, 7S, 4S) and their byte rotations. The final stage G runs
// 32 extra ROR3/CMIX/SMIX rounds then 13 rounds of four ROR9/ROR8 + SMIX steps.
namespace {

struct FugueTables {
    u32 mt[4][256];
    FugueTables() {
        const u8* S = aes_sbox();
        for (int x = 0; x < 256; ++x) {
            const u8 s = S[x];
            const u32 v = (u32(s) << 24) | (u32(s) << 16) | (u32(gmul(s, 7)) << 8) | u32(gmul(s, 4));
            for (int k = 0; k < 4; ++k) mt[k][x] = k ? rotr32(v, 8 * k) : v;
        }
    }
};

void fugue_smix(const FugueTables& T, u32& x0, u32& x1, u32& x2, u32& x3) {
    u32 x[4] = {x0, x1, x2, x3}, c[4] = {0, 0, 0, 0}, r[4] = {0, 0, 0, 0};
    for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 4; ++k) {
            const u32 t = T.mt[k][(x[j] >> (24 - 8 * k)) & 0xFF];
            c[j] ^= t;
            if (k != j) r[k] ^= t;
        }
    x0 = ((c[0] ^ r[0]) & 0xFF000000u) | ((c[1] ^ r[1]) & 0x00FF0000u) | ((c[2] ^ r[2]) & 0x0000FF00u) |
         ((c[3] ^ r[3]) & 0x000000FFu);
    x1 = ((c[1] ^ (r[0] << 8)) & 0xFF000000u) | ((c[2] ^ (r[1] << 8)) & 0x00FF0000u) |
         ((c[3] ^ (r[2] << 8)) & 0x0000FF00u) | ((c[0] ^ (r[3] >> 24)) & 0x000000FFu);
    x2 = ((c[2] ^ (r[0] << 16)) & 0xFF000000u) | ((c[3] ^ (r[1] << 16)) & 0x00FF0000u) |
         ((c[0] ^ (r[2] >> 16)) & 0x0000FF00u) | ((c[1] ^ (r[3] >> 16)) & 0x000000FFu);
    x3 = ((c[3] ^ (r[0] << 24)) & 0xFF000000u) | ((c[0] ^ (r[1] >> 8)) & 0x00FF0000u) |
         ((c[1] ^ (r[2] >> 8)) & 0x0000FF00u) | ((c[2] ^ (r[3] >> 8)) & 0x000000FFu);
}

// The 36 columns as a ring: logical column i is R[(i + off) % 36], so the ROR3 / ROR8 / ROR9
// rotations are offset updates instead of 36-word moves.
struct Fugue {
    u32 R[36];
    int off = 0;
    const FugueTables& T;
    explicit Fugue(const FugueTables& t) : T(t) {}
    u32& S(int i) {
        const int j = i + off;
        return R[j >= 36 ? j - 36 : j];
    }
    void ror(int n) { off = off >= n ? off - n : off - n + 36; }
    void smix() { fugue_smix(T, S(0), S(1), S(2), S(3)); }
    void cmix_sub() {
        ror(3);
        S(0) ^= S(4); S(1) ^= S(5); S(2) ^= S(6);
        S(18) ^= S(4); S(19) ^= S(5); S(20) ^= S(6);
        smix();
    }
    void word(u32 I) {
        S(22) ^= S(0);
        S(0) = I;
        S(8) ^= S(0);
        S(1) ^= S(24);
        S(4) ^= S(27);
        S(7) ^= S(30);
        for (int k = 0; k < 4; ++k) cmix_sub();
    }
};

}  // namespace

Hash512 fugue512(const u8* data, size_t n) {
    static const FugueTables T;
    static const u32 kIV[16] = {0x8807a57e, 0xe616af75, 0xc5d3e4db, 0xac9ab027, 0xd915f117, 0xb6eecc54,
                                0x06e8020b, 0x4a92efd1, 0xaac6e2c9, 0xddb21398, 0xcae65838, 0x437f203f,
                                0x25ea78e7, 0x951fddd6, 0xda6ed11d, 0xe13e3567};
    Fugue f(T);
    std::memset(f.R, 0, sizeof f.R);
    std::memcpy(f.R + 20, kIV, sizeof kIV);
    const u64 bits = u64(n) * 8;
    for (; n >= 4; n -= 4, data += 4) f.word(load_be32(data));
    if (n) {
        u8 w[4] = {0};
        std::memcpy(w, data, n);
        f.word(load_be32(w));
    }
    f.word(u32(bits >> 32));
    f.word(u32(bits));
    for (int i = 0; i < 32; ++i) f.cmix_sub();
    static const int kG[4][4] = {{4, 9, 18, 27}, {4, 10, 18, 27}, {4, 10, 19, 27}, {4, 10, 19, 28}};
    for (int i = 0; i < 13; ++i)
        for (int k = 0; k < 4; ++k) {
            for (int j = 0; j < 4; ++j) f.S(kG[k][j]) ^= f.S(0);
            f.ror(k == 3 ? 8 : 9);
            f.smix();
        }
    for (int j = 0; j < 4; ++j) f.S(kG[0][j]) ^= f.S(0);
    static const int kOut[16] = {1, 2, 3, 4, 9, 10, 11, 12, 18, 19, 20, 21, 27, 28, 29, 30};
    Hash512 out;
    for (int i = 0; i < 16; ++i) store_be32(out.bytes + 4 * i, f.S(kOut[i]));
    return out;
}

}  // namespace nodexa
