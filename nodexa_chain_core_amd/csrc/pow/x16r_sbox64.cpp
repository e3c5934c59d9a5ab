// X16R byte-substitution primitives with 64-bit table lookups: Whirlpool and Tiger.
//
// Parity: sph_whirlpool (slot 14 of HashX16R, src/hash.h:428-432) and sph_tiger
// (the X16RV2 pre-hash, src/hash.h:531,545,594). Both S-box sets are *derived*
// at first use from their published constructions rather than stored:
//   * Whirlpool (ISO/IEC 10118-3): the 8-bit S-box is built from the E, E^-1
//     and R 4-bit mini-boxes; the diffusion layer is the circulant MDS matrix
//     cir(1,1,4,1,8,5,2,9) over GF(2^8)/0x11D; 10 rounds, Miyaguchi-Preneel.
//   * Tiger (Anderson & Biham, 1995): the four 256 x 64-bit S-boxes come from
//     the authors' generator — identity tables shuffled for 5 passes by bytes of
//     the Tiger state, re-compressed (with the tables under construction) over
//     the 64-byte title string every third step.
#include "x16r_prims.hpp"

namespace nodexa {

// ================================================================ Whirlpool
namespace {

u8 gf_mul_11d(u8 a, u8 b) {
    u8 r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = u8((a << 1) ^ ((a & 0x80) ? 0x1D : 0));
        b >>= 1;
    }
    return r;
}

struct WhirlTables {
    u8 S[256];
    u64 T[8][256];  // T[k][x] = row contribution of S[x] in column position k (after theta)
    u64 rc[11];
    WhirlTables() {
        const u8 E[16] = {0x1, 0xB, 0x9, 0xC, 0xD, 0x6, 0xF, 0x3, 0xE, 0x8, 0x7, 0x4, 0xA, 0x2, 0x5, 0x0};
        const u8 R[16] = {0x7, 0xC, 0xB, 0xD, 0xE, 0x4, 0x9, 0xF, 0x6, 0x3, 0x8, 0xA, 0x2, 0x5, 0x1, 0x0};
        u8 Ei[16];
        for (int i = 0; i < 16; ++i) Ei[E[i]] = u8(i);
        for (int u = 0; u < 256; ++u) {
            const u8 a = E[u >> 4], b = Ei[u & 15], c = R[a ^ b];
            S[u] = u8((E[a ^ c] << 4) | Ei[b ^ c]);
        }
        const u8 cir[8] = {1, 1, 4, 1, 8, 5, 2, 9};
        // Row vector a (8 bytes) times C, C[k][j] = cir[(j - k) & 7]. A byte at column k
        // contributes S[x]*C[k][j] to output column j; pack output bytes LE in j.
        for (int k = 0; k < 8; ++k)
            for (int x = 0; x < 256; ++x) {
                u64 v = 0;
                for (int j = 0; j < 8; ++j) v |= u64(gf_mul_11d(S[x], cir[(j - k) & 7])) << (8 * j);
                T[k][x] = v;
            }
        rc[0] = 0;
        for (int r = 1; r <= 10; ++r) {
            u64 v = 0;
            for (int j = 0; j < 8; ++j) v |= u64(S[8 * (r - 1) + j]) << (8 * j);
            rc[r] = v;
        }
    }
};

const WhirlTables& whirl() {
    static const WhirlTables t;
    return t;
}

// rho[k](a) = sigma[k] . theta . pi . gamma over 8 rows (u64, byte j = column j).
void whirl_round(const WhirlTables& t, const u64 a[8], const u64 k[8], u64 out[8]) {
    for (int i = 0; i < 8; ++i) {
        u64 v = k[i];
        // pi: b[i][j] = a[(i - j) & 7][j]; gamma+theta via the tables
        for (int j = 0; j < 8; ++j) v ^= t.T[j][u8(a[(i - j) & 7] >> (8 * j))];
        out[i] = v;
    }
}

void whirl_compress(u64 H[8], const u8 blk[64]) {
    const WhirlTables& t = whirl();
    u64 K[8], st[8], m[8], tmp[8];
    for (int i = 0; i < 8; ++i) {
        m[i] = load_le64(blk + 8 * i);
        K[i] = H[i];
        st[i] = m[i] ^ K[i];
    }
    for (int r = 1; r <= 10; ++r) {
        u64 c[8] = {t.rc[r], 0, 0, 0, 0, 0, 0, 0};
        whirl_round(t, K, c, tmp);
        std::memcpy(K, tmp, sizeof K);
        whirl_round(t, st, K, tmp);
        std::memcpy(st, tmp, sizeof st);
    }
    for (int i = 0; i < 8; ++i) H[i] ^= st[i] ^ m[i];
}

}  // namespace

Hash512 whirlpool512(const u8* data, size_t n) {
    u64 H[8] = {0};
    const u64 bits = u64(n) * 8;
    for (; n >= 64; n -= 64, data += 64) whirl_compress(H, data);
    u8 buf[128] = {0};
    std::memcpy(buf, data, n);
    buf[n] = 0x80;
    const size_t len = n < 32 ? 64 : 128;  // 256-bit length field at the end
    store_be64(buf + len - 8, bits);
    whirl_compress(H, buf);
    if (len == 128) whirl_compress(H, buf + 64);
    Hash512 out;
    for (int i = 0; i < 8; ++i) store_le64(out.bytes + 8 * i, H[i]);
    return out;
}

// ================================================================ Tiger (Tiger/192, 0x01 padding)
namespace {

struct TigerTables {
    u64 t[4][256];
    TigerTables();
};

const TigerTables& tiger_tables();

void tiger_compress(const u64 (&T)[4][256], const u64 xin[8], u64 st[3]) {
    u64 a = st[0], b = st[1], c = st[2], x[8];
    std::memcpy(x, xin, sizeof x);
    auto rnd = [&](u64& A, u64& B, u64& C, u64 xv, u64 mul) {
        C ^= xv;
        A -= T[0][u8(C)] ^ T[1][u8(C >> 16)] ^ T[2][u8(C >> 32)] ^ T[3][u8(C >> 48)];
        B += T[3][u8(C >> 8)] ^ T[2][u8(C >> 24)] ^ T[1][u8(C >> 40)] ^ T[0][u8(C >> 56)];
        B *= mul;
    };
    auto pass = [&](u64& A, u64& B, u64& C, u64 mul) {
        rnd(A, B, C, x[0], mul); rnd(B, C, A, x[1], mul); rnd(C, A, B, x[2], mul); rnd(A, B, C, x[3], mul);
        rnd(B, C, A, x[4], mul); rnd(C, A, B, x[5], mul); rnd(A, B, C, x[6], mul); rnd(B, C, A, x[7], mul);
    };
    auto schedule = [&]() {
        x[0] -= x[7] ^ 0xA5A5A5A5A5A5A5A5ULL; x[1] ^= x[0]; x[2] += x[1]; x[3] -= x[2] ^ ((~x[1]) << 19);
        x[4] ^= x[3]; x[5] += x[4]; x[6] -= x[5] ^ ((~x[4]) >> 23); x[7] ^= x[6];
        x[0] += x[7]; x[1] -= x[0] ^ ((~x[7]) << 19); x[2] ^= x[1]; x[3] += x[2];
        x[4] -= x[3] ^ ((~x[2]) >> 23); x[5] ^= x[4]; x[6] += x[5]; x[7] -= x[6] ^ 0x0123456789ABCDEFULL;
    };
    pass(a, b, c, 5);
    schedule();
    pass(c, a, b, 7);
    schedule();
    pass(b, c, a, 9);
    st[0] = a ^ st[0];
    st[1] = b - st[1];
    st[2] = c + st[2];
}

TigerTables::TigerTables() {
    static const char title[] = "Tiger - A Fast New Hash Function, by Ross Anderson and Eli Biham";
    static_assert(sizeof(title) == 65, "title is one 64-byte block");
    u64 msg[8];
    for (int i = 0; i < 8; ++i) msg[i] = load_le64(reinterpret_cast<const u8*>(title) + 8 * i);
    u8* bytes = reinterpret_cast<u8*>(&t[0][0]);  // 1024 entries x 8 bytes (little-endian host)
    for (int i = 0; i < 1024; ++i)
        for (int col = 0; col < 8; ++col) bytes[8 * i + col] = u8(i);
    u64 st[3] = {0x0123456789ABCDEFULL, 0xFEDCBA9876543210ULL, 0xF096A5B4C3B2E187ULL};
    int abc = 2;
    for (int pass = 0; pass < 5; ++pass)
        for (int i = 0; i < 256; ++i)
            for (int sb = 0; sb < 1024; sb += 256) {
                if (++abc == 3) {
                    abc = 0;
                    tiger_compress(t, msg, st);
                }
                for (int col = 0; col < 8; ++col) {
                    const int j = u8(st[abc] >> (8 * col));
                    std::swap(bytes[8 * (sb + i) + col], bytes[8 * (sb + j) + col]);
                }
            }
}

const TigerTables& tiger_tables() {
    static const TigerTables tt;
    return tt;
}

}  // namespace

Hash512 tiger192_padded(const u8* data, size_t n) {
    const auto& T = tiger_tables().t;
    u64 st[3] = {0x0123456789ABCDEFULL, 0xFEDCBA9876543210ULL, 0xF096A5B4C3B2E187ULL};
    u64 x[8];
    const u64 bits = u64(n) * 8;
    for (; n >= 64; n -= 64, data += 64) {
        for (int i = 0; i < 8; ++i) x[i] = load_le64(data + 8 * i);
        tiger_compress(T, x, st);
    }
    u8 buf[128] = {0};
    std::memcpy(buf, data, n);
    buf[n] = 0x01;
    const size_t len = n < 56 ? 64 : 128;
    store_le64(buf + len - 8, bits);
    for (size_t off = 0; off < len; off += 64) {
        for (int i = 0; i < 8; ++i) x[i] = load_le64(buf + off + 8 * i);
        tiger_compress(T, x, st);
    }
    Hash512 out;  // zero-filled: the reference hashes into a zeroed uint512 (src/hash.h:531)
    for (int i = 0; i < 3; ++i) store_le64(out.bytes + 8 * i, st[i]);
    return out;
}

}  // namespace nodexa
