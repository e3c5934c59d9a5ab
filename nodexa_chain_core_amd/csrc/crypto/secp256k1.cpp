// secp256k1 host arithmetic: see secp256k1.hpp. Field and scalar elements are 4 x 64-bit limbs
// multiplied through unsigned __int128 and reduced with the special forms of p and n
// (2^256 = 0x1000003D1 mod p, 2^256 = 2^256 - n mod n).
#include "secp256k1.hpp"

#include <cstring>
#include <vector>

#include "hashes.hpp"

namespace nodexa::secp {

using u128 = unsigned __int128;

namespace {

constexpr u64 kP[4] = {0xFFFFFFFEFFFFFC2FULL, ~0ULL, ~0ULL, ~0ULL};
constexpr u64 kPC = 0x1000003D1ULL;  // 2^256 - p
constexpr u64 kN[4] = {0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, ~0ULL};
constexpr u64 kNC[3] = {0x402DA1732FC9BEBFULL, 0x4551231950B75FC4ULL, 1ULL};  // 2^256 - n
constexpr u64 kNHalf[4] = {0xDFE92F46681B20A0ULL, 0x5D576E7357A4501DULL, 0xFFFFFFFFFFFFFFFFULL,
                           0x7FFFFFFFFFFFFFFFULL};

bool geq(const u64 a[4], const u64 b[4]) {
    for (int i = 3; i >= 0; --i) {
        if (a[i] != b[i]) return a[i] > b[i];
    }
    return true;
}

// r = a - b (4 limbs), returns the borrow
u64 sub4(u64 r[4], const u64 a[4], const u64 b[4]) {
    u64 borrow = 0;
    for (int i = 0; i < 4; ++i) {
        const u128 d = (u128)a[i] - b[i] - borrow;
        r[i] = (u64)d;
        borrow = (u64)(d >> 64) & 1;
    }
    return borrow;
}

// r = a + b (4 limbs), returns the carry
u64 add4(u64 r[4], const u64 a[4], const u64 b[4]) {
    u64 carry = 0;
    for (int i = 0; i < 4; ++i) {
        const u128 s = (u128)a[i] + b[i] + carry;
        r[i] = (u64)s;
        carry = (u64)(s >> 64);
    }
    return carry;
}

void mul4x4(const u64 a[4], const u64 b[4], u64 t[8]) {
    for (int i = 0; i < 8; ++i) t[i] = 0;
    for (int i = 0; i < 4; ++i) {
        u64 carry = 0;
        for (int j = 0; j < 4; ++j) {
            const u128 m = (u128)a[i] * b[j] + t[i + j] + carry;
            t[i + j] = (u64)m;
            carry = (u64)(m >> 64);
        }
        t[i + 4] = carry;
    }
}

// 512-bit t mod p
Fe fe_reduce512(const u64 t[8]) {
    // r = lo + hi * PC (hi * PC < 2^290): five limbs
    u64 r[5];
    u64 carry = 0;
    for (int i = 0; i < 4; ++i) {
        const u128 m = (u128)t[4 + i] * kPC + t[i] + carry;
        r[i] = (u64)m;
        carry = (u64)(m >> 64);
    }
    r[4] = carry;
    // fold r[4] * PC (< 2^98) into the low four limbs
    u128 m = (u128)r[4] * kPC + r[0];
    r[0] = (u64)m;
    u64 c = (u64)(m >> 64);
    for (int i = 1; i < 4 && c; ++i) {
        const u128 s = (u128)r[i] + c;
        r[i] = (u64)s;
        c = (u64)(s >> 64);
    }
    if (c) {  // wrapped past 2^256 once more: add PC (cannot carry again)
        const u128 s = (u128)r[0] + kPC;
        r[0] = (u64)s;
        u64 cc = (u64)(s >> 64);
        for (int i = 1; i < 4 && cc; ++i) {
            const u128 t2 = (u128)r[i] + cc;
            r[i] = (u64)t2;
            cc = (u64)(t2 >> 64);
        }
    }
    Fe out;
    std::memcpy(out.v, r, 32);
    if (geq(out.v, kP)) sub4(out.v, out.v, kP);
    return out;
}

// value (nl <= 8 limbs) mod n: fold hi * (2^256 - n) into lo until 4 limbs remain (fixed-size,
// no allocation: 512 -> 386 -> 259 -> 256 bits)
Scalar sc_reduce(const u64* t, int nl) {
    u64 v[9] = {0};
    for (int i = 0; i < nl; ++i) v[i] = t[i];
    int n = nl;
    while (n > 4 && v[n - 1] == 0) --n;
    while (n > 4) {
        const int nh = n - 4;
        const int rn = (nh + 3 > 4 ? nh + 3 : 4) + 1;
        u64 r[9] = {v[0], v[1], v[2], v[3], 0, 0, 0, 0, 0};
        for (int i = 0; i < nh; ++i) {
            u64 carry = 0;
            for (int j = 0; j < 3; ++j) {
                const u128 m = (u128)v[4 + i] * kNC[j] + r[i + j] + carry;
                r[i + j] = (u64)m;
                carry = (u64)(m >> 64);
            }
            for (int k = i + 3; carry && k < rn; ++k) {
                const u128 s2 = (u128)r[k] + carry;
                r[k] = (u64)s2;
                carry = (u64)(s2 >> 64);
            }
        }
        for (int i = 0; i < 9; ++i) v[i] = r[i];
        n = rn;
        while (n > 4 && v[n - 1] == 0) --n;
    }
    Scalar s;
    for (int i = 0; i < 4; ++i) s.v[i] = v[i];
    while (geq(s.v, kN)) sub4(s.v, s.v, kN);
    return s;
}

// 512-bit square: the six cross products once, doubled, plus the four squares
void sqr4(const u64 a[4], u64 t[8]) {
    u64 c[8] = {0};
    for (int i = 0; i < 4; ++i) {
        u64 carry = 0;
        for (int j = i + 1; j < 4; ++j) {
            const u128 m = (u128)a[i] * a[j] + c[i + j] + carry;
            c[i + j] = (u64)m;
            carry = (u64)(m >> 64);
        }
        c[i + 4] = carry;
    }
    u64 top = 0;
    for (int i = 0; i < 8; ++i) {  // c *= 2
        const u64 nt = c[i] >> 63;
        c[i] = (c[i] << 1) | top;
        top = nt;
    }
    u64 carry = 0;
    for (int i = 0; i < 4; ++i) {
        const u128 sq = (u128)a[i] * a[i];
        u128 lo = (u128)c[2 * i] + (u64)sq + carry;
        t[2 * i] = (u64)lo;
        u128 hi = (u128)c[2 * i + 1] + (u64)(sq >> 64) + (u64)(lo >> 64);
        t[2 * i + 1] = (u64)hi;
        carry = (u64)(hi >> 64);
    }
}

void be_to_limbs(const u8 b[32], u64 v[4]) {
    for (int i = 0; i < 4; ++i) {
        u64 x = 0;
        for (int k = 0; k < 8; ++k) x = (x << 8) | b[(3 - i) * 8 + k];
        v[i] = x;
    }
}

void limbs_to_be(const u64 v[4], u8 b[32]) {
    for (int i = 0; i < 4; ++i)
        for (int k = 0; k < 8; ++k) b[(3 - i) * 8 + k] = (u8)(v[i] >> (56 - 8 * k));
}

Fe fe_small(u64 x) {
    Fe r;
    r.v[0] = x;
    return r;
}


}  // namespace

// ------------------------------------------------------------------ field
Fe fe_from_be(const u8 b[32], bool* overflow) {
    Fe r;
    be_to_limbs(b, r.v);
    const bool of = geq(r.v, kP);
    if (of) sub4(r.v, r.v, kP);
    if (overflow) *overflow = of;
    return r;
}

void fe_to_be(const Fe& a, u8 out[32]) { limbs_to_be(a.v, out); }

Fe fe_add(const Fe& a, const Fe& b) {
    Fe r;
    const u64 c = add4(r.v, a.v, b.v);
    if (c || geq(r.v, kP)) sub4(r.v, r.v, kP);  // mod 2^256 this adds PC when c is set
    return r;
}

Fe fe_sub(const Fe& a, const Fe& b) {
    Fe r;
    if (sub4(r.v, a.v, b.v)) add4(r.v, r.v, kP);
    return r;
}

Fe fe_neg(const Fe& a) { return fe_sub(Fe{}, a); }

Fe fe_mul(const Fe& a, const Fe& b) {
    u64 t[8];
    mul4x4(a.v, b.v, t);
    return fe_reduce512(t);
}

Fe fe_sqr(const Fe& a) {
    u64 t[8];
    sqr4(a.v, t);
    return fe_reduce512(t);
}

bool fe_eq(const Fe& a, const Fe& b) { return std::memcmp(a.v, b.v, 32) == 0; }
bool fe_is_zero(const Fe& a) { return (a.v[0] | a.v[1] | a.v[2] | a.v[3]) == 0; }
bool fe_is_odd(const Fe& a) { return a.v[0] & 1; }

static Fe fe_pow(const Fe& a, const u64 e[4]) {
    Fe r = fe_small(1);
    for (int i = 255; i >= 0; --i) {
        r = fe_sqr(r);
        if ((e[i / 64] >> (i % 64)) & 1) r = fe_mul(r, a);
    }
    return r;
}

Fe fe_inv(const Fe& a) {
    const u64 e[4] = {kP[0] - 2, kP[1], kP[2], kP[3]};
    return fe_pow(a, e);
}

bool fe_sqrt(const Fe& a, Fe& r) {
    // (p + 1) / 4
    const u64 e[4] = {0xFFFFFFFFBFFFFF0CULL, ~0ULL, ~0ULL, 0x3FFFFFFFFFFFFFFFULL};
    r = fe_pow(a, e);
    return fe_eq(fe_sqr(r), a);
}

// ------------------------------------------------------------------ scalar
Scalar sc_from_be(const u8 b[32], bool* overflow) {
    Scalar r;
    be_to_limbs(b, r.v);
    const bool of = geq(r.v, kN);
    if (of) sub4(r.v, r.v, kN);
    if (overflow) *overflow = of;
    return r;
}

void sc_to_be(const Scalar& a, u8 out[32]) { limbs_to_be(a.v, out); }

Scalar sc_add(const Scalar& a, const Scalar& b) {
    Scalar r;
    const u64 c = add4(r.v, a.v, b.v);
    if (c || geq(r.v, kN)) sub4(r.v, r.v, kN);
    return r;
}

Scalar sc_neg(const Scalar& a) {
    if (a.is_zero()) return a;
    Scalar r;
    sub4(r.v, kN, a.v);
    return r;
}

Scalar sc_mul(const Scalar& a, const Scalar& b) {
    u64 t[8];
    mul4x4(a.v, b.v, t);
    return sc_reduce(t, 8);
}

Scalar sc_inv(const Scalar& a) {
    const u64 e[4] = {kN[0] - 2, kN[1], kN[2], kN[3]};
    Scalar r;
    r.v[0] = 1;
    for (int i = 255; i >= 0; --i) {
        r = sc_mul(r, r);
        if ((e[i / 64] >> (i % 64)) & 1) r = sc_mul(r, a);
    }
    return r;
}

bool sc_is_high(const Scalar& a) { return !geq(kNHalf, a.v); }

// ------------------------------------------------------------------ group
const Ge& generator() {
    static const Ge g = [] {
        static const u8 gx[32] = {0x79, 0xBE, 0x66, 0x7E, 0xF9, 0xDC, 0xBB, 0xAC, 0x55, 0xA0, 0x62,
                                  0x95, 0xCE, 0x87, 0x0B, 0x07, 0x02, 0x9B, 0xFC, 0xDB, 0x2D, 0xCE,
                                  0x28, 0xD9, 0x59, 0xF2, 0x81, 0x5B, 0x16, 0xF8, 0x17, 0x98};
        static const u8 gy[32] = {0x48, 0x3A, 0xDA, 0x77, 0x26, 0xA3, 0xC4, 0x65, 0x5D, 0xA4, 0xFB,
                                  0xFC, 0x0E, 0x11, 0x08, 0xA8, 0xFD, 0x17, 0xB4, 0x48, 0xA6, 0x85,
                                  0x54, 0x19, 0x9C, 0x47, 0xD0, 0x8F, 0xFB, 0x10, 0xD4, 0xB8};
        Ge p;
        p.x = fe_from_be(gx);
        p.y = fe_from_be(gy);
        p.inf = false;
        return p;
    }();
    return g;
}

Gej gej_from_ge(const Ge& a) {
    Gej r;
    r.inf = a.inf;
    if (!a.inf) {
        r.x = a.x;
        r.y = a.y;
        r.z = fe_small(1);
    }
    return r;
}

Ge ge_from_gej(const Gej& a) {
    Ge r;
    if (a.inf) return r;
    const Fe zi = fe_inv(a.z), zi2 = fe_sqr(zi), zi3 = fe_mul(zi2, zi);
    r.x = fe_mul(a.x, zi2);
    r.y = fe_mul(a.y, zi3);
    r.inf = false;
    return r;
}

bool ge_on_curve(const Ge& a) {
    if (a.inf) return false;
    const Fe y2 = fe_sqr(a.y), x3 = fe_mul(fe_sqr(a.x), a.x);
    return fe_eq(y2, fe_add(x3, fe_small(7)));
}

Gej gej_double(const Gej& a) {
    if (a.inf || fe_is_zero(a.y)) return Gej{};
    const Fe A = fe_sqr(a.x), B = fe_sqr(a.y), C = fe_sqr(B);
    const Fe xb = fe_add(a.x, B);
    Fe D = fe_sub(fe_sub(fe_sqr(xb), A), C);
    D = fe_add(D, D);
    const Fe E = fe_add(fe_add(A, A), A), F = fe_sqr(E);
    Gej r;
    r.x = fe_sub(F, fe_add(D, D));
    const Fe C2 = fe_add(C, C), C4 = fe_add(C2, C2), C8 = fe_add(C4, C4);
    r.y = fe_sub(fe_mul(E, fe_sub(D, r.x)), C8);
    const Fe yz = fe_mul(a.y, a.z);
    r.z = fe_add(yz, yz);
    r.inf = false;
    return r;
}

Gej gej_add(const Gej& a, const Gej& b) {
    if (a.inf) return b;
    if (b.inf) return a;
    const Fe z1z1 = fe_sqr(a.z), z2z2 = fe_sqr(b.z);
    const Fe u1 = fe_mul(a.x, z2z2), u2 = fe_mul(b.x, z1z1);
    const Fe s1 = fe_mul(fe_mul(a.y, b.z), z2z2), s2 = fe_mul(fe_mul(b.y, a.z), z1z1);
    const Fe h = fe_sub(u2, u1);
    Fe rr = fe_sub(s2, s1);
    if (fe_is_zero(h)) return fe_is_zero(rr) ? gej_double(a) : Gej{};
    rr = fe_add(rr, rr);
    const Fe h2 = fe_add(h, h), i = fe_sqr(h2), j = fe_mul(h, i), v = fe_mul(u1, i);
    Gej r;
    r.x = fe_sub(fe_sub(fe_sqr(rr), j), fe_add(v, v));
    const Fe s1j = fe_mul(s1, j);
    r.y = fe_sub(fe_mul(rr, fe_sub(v, r.x)), fe_add(s1j, s1j));
    r.z = fe_mul(fe_sub(fe_sub(fe_sqr(fe_add(a.z, b.z)), z1z1), z2z2), h);
    r.inf = false;
    return r;
}

Gej gej_add_ge(const Gej& a, const Ge& b) {
    if (b.inf) return a;
    if (a.inf) return gej_from_ge(b);
    const Fe z1z1 = fe_sqr(a.z);
    const Fe u2 = fe_mul(b.x, z1z1), s2 = fe_mul(fe_mul(b.y, a.z), z1z1);
    const Fe h = fe_sub(u2, a.x);
    Fe rr = fe_sub(s2, a.y);
    if (fe_is_zero(h)) return fe_is_zero(rr) ? gej_double(a) : Gej{};
    rr = fe_add(rr, rr);
    const Fe hh = fe_sqr(h), i = fe_add(fe_add(hh, hh), fe_add(hh, hh)), j = fe_mul(h, i), v = fe_mul(a.x, i);
    Gej r;
    r.x = fe_sub(fe_sub(fe_sqr(rr), j), fe_add(v, v));
    const Fe yj = fe_mul(a.y, j);
    r.y = fe_sub(fe_mul(rr, fe_sub(v, r.x)), fe_add(yj, yj));
    r.z = fe_sub(fe_sub(fe_sqr(fe_add(a.z, h)), z1z1), hh);
    r.inf = false;
    return r;
}

namespace {

// table[i][j] = j * 16^i * G (affine), i < 64, j < 16: k*G is 64 mixed additions.
struct GenTable {
    Ge t[64][16];
    GenTable() {
        Gej base = gej_from_ge(generator());
        for (int i = 0; i < 64; ++i) {
            Gej acc;  // infinity
            t[i][0] = Ge{};
            for (int j = 1; j < 16; ++j) {
                acc = gej_add(acc, base);
                t[i][j] = ge_from_gej(acc);
            }
            for (int k = 0; k < 4; ++k) base = gej_double(base);
        }
    }
};

const GenTable& gen_table() {
    static const GenTable* t = new GenTable();  // built once, thread-safe static init
    return *t;
}

int nibble(const Scalar& k, int i) { return (int)((k.v[i / 16] >> (4 * (i % 16))) & 15); }

}  // namespace

Gej mul_gen(const Scalar& k) {
    const GenTable& t = gen_table();
    Gej r;
    for (int i = 0; i < 64; ++i) {
        const int nb = nibble(k, i);
        if (nb) r = gej_add_ge(r, t.t[i][nb]);
    }
    return r;
}

namespace {

// width-5 NAF of k: digits in {0, +-1, +-3, ..., +-15}, least significant first
int wnaf5(const Scalar& k, int8_t out[258]) {
    u64 v[5] = {k.v[0], k.v[1], k.v[2], k.v[3], 0};
    int len = 0;
    while (v[0] | v[1] | v[2] | v[3] | v[4]) {
        int d = 0;
        if (v[0] & 1) {
            d = int(v[0] & 31);
            if (d >= 16) d -= 32;
            if (d > 0) {  // v -= d
                u64 b = u64(d);
                for (int i = 0; i < 5 && b; ++i) {
                    const u64 o = v[i];
                    v[i] -= b;
                    b = v[i] > o;
                }
            } else {  // v += -d
                u64 c = u64(-d);
                for (int i = 0; i < 5 && c; ++i) {
                    v[i] += c;
                    c = v[i] < c;
                }
            }
        }
        out[len++] = int8_t(d);
        for (int i = 0; i < 4; ++i) v[i] = (v[i] >> 1) | (v[i + 1] << 63);
        v[4] >>= 1;
    }
    return len;
}

Gej gej_neg(const Gej& a) {
    Gej r = a;
    if (!a.inf) r.y = fe_neg(a.y);
    return r;
}

}  // namespace

Gej mul(const Ge& p, const Scalar& k) {
    if (p.inf || k.is_zero()) return Gej{};
    Gej tab[8];  // P, 3P, ..., 15P
    tab[0] = gej_from_ge(p);
    const Gej p2 = gej_double(tab[0]);
    for (int j = 1; j < 8; ++j) tab[j] = gej_add(tab[j - 1], p2);
    int8_t naf[258];
    const int len = wnaf5(k, naf);
    Gej r;
    for (int i = len - 1; i >= 0; --i) {
        r = gej_double(r);
        const int d = naf[i];
        if (d > 0) r = gej_add(r, tab[d >> 1]);
        else if (d < 0) r = gej_add(r, gej_neg(tab[(-d) >> 1]));
    }
    return r;
}

Gej mul_double(const Scalar& a, const Ge& p, const Scalar& b) { return gej_add(mul(p, a), mul_gen(b)); }

// ------------------------------------------------------------------ keys and signatures
bool pubkey_parse(const u8* in, size_t len, Ge& out) {
    out = Ge{};
    if (len == 33 && (in[0] == 2 || in[0] == 3)) {
        bool of = false;
        const Fe x = fe_from_be(in + 1, &of);
        if (of) return false;
        const Fe rhs = fe_add(fe_mul(fe_sqr(x), x), fe_small(7));
        Fe y;
        if (!fe_sqrt(rhs, y)) return false;
        if (fe_is_odd(y) != (in[0] == 3)) y = fe_neg(y);
        out.x = x;
        out.y = y;
        out.inf = false;
        return true;
    }
    if (len == 65 && (in[0] == 4 || in[0] == 6 || in[0] == 7)) {
        bool ofx = false, ofy = false;
        out.x = fe_from_be(in + 1, &ofx);
        out.y = fe_from_be(in + 33, &ofy);
        out.inf = false;
        if (ofx || ofy) return false;
        if (in[0] != 4 && fe_is_odd(out.y) != (in[0] == 7)) return false;  // hybrid: parity must match
        return ge_on_curve(out);
    }
    return false;
}

size_t pubkey_serialize(const Ge& p, bool compressed, u8 out[65]) {
    if (compressed) {
        out[0] = fe_is_odd(p.y) ? 3 : 2;
        fe_to_be(p.x, out + 1);
        return 33;
    }
    out[0] = 4;
    fe_to_be(p.x, out + 1);
    fe_to_be(p.y, out + 33);
    return 65;
}

bool seckey_valid(const u8 key[32]) {
    bool of = false;
    const Scalar k = sc_from_be(key, &of);
    return !of && !k.is_zero();
}

bool pubkey_create(const u8 key[32], Ge& out) {
    if (!seckey_valid(key)) return false;
    out = ge_from_gej(mul_gen(sc_from_be(key)));
    return true;
}

bool sig_parse_der_lax(const u8* in, size_t len, Scalar& r, Scalar& s) {
    r = Scalar{};
    s = Scalar{};
    size_t pos = 0;
    if (pos == len || in[pos] != 0x30) return false;
    ++pos;
    if (pos == len) return false;
    size_t lenbyte = in[pos++];
    if (lenbyte & 0x80) {
        lenbyte -= 0x80;
        if (lenbyte > len - pos) return false;
        pos += lenbyte;
    }
    size_t rpos = 0, rlen = 0, spos = 0, slen = 0;
    for (int which = 0; which < 2; ++which) {
        if (pos == len || in[pos] != 0x02) return false;
        ++pos;
        if (pos == len) return false;
        lenbyte = in[pos++];
        size_t ilen;
        if (lenbyte & 0x80) {
            lenbyte -= 0x80;
            if (lenbyte > len - pos) return false;
            while (lenbyte > 0 && in[pos] == 0) {
                ++pos;
                --lenbyte;
            }
            if (lenbyte >= sizeof(size_t)) return false;
            ilen = 0;
            while (lenbyte > 0) {
                ilen = (ilen << 8) + in[pos];
                ++pos;
                --lenbyte;
            }
        } else {
            ilen = lenbyte;
        }
        if (ilen > len - pos) return false;
        (which ? spos : rpos) = pos;
        (which ? slen : rlen) = ilen;
        pos += ilen;
    }
    while (rlen > 0 && in[rpos] == 0) {
        --rlen;
        ++rpos;
    }
    while (slen > 0 && in[spos] == 0) {
        --slen;
        ++spos;
    }
    u8 tmp[64] = {0};
    bool overflow = rlen > 32 || slen > 32;
    if (!overflow) {
        std::memcpy(tmp + 32 - rlen, in + rpos, rlen);
        std::memcpy(tmp + 64 - slen, in + spos, slen);
        bool of1 = false, of2 = false;
        r = sc_from_be(tmp, &of1);
        s = sc_from_be(tmp + 32, &of2);
        overflow = of1 || of2;
    }
    if (overflow) {  // a parsed but never-valid signature
        r = Scalar{};
        s = Scalar{};
    }
    return true;
}

size_t sig_serialize_der(const Scalar& r, const Scalar& s, u8 out[72]) {
    u8 rb[33], sb[33];
    rb[0] = sb[0] = 0;
    sc_to_be(r, rb + 1);
    sc_to_be(s, sb + 1);
    const u8* rp = rb;
    const u8* sp = sb;
    size_t rl = 33, sl = 33;
    while (rl > 1 && rp[0] == 0 && !(rp[1] & 0x80)) {
        ++rp;
        --rl;
    }
    while (sl > 1 && sp[0] == 0 && !(sp[1] & 0x80)) {
        ++sp;
        --sl;
    }
    size_t n = 0;
    out[n++] = 0x30;
    out[n++] = (u8)(4 + rl + sl);
    out[n++] = 0x02;
    out[n++] = (u8)rl;
    std::memcpy(out + n, rp, rl);
    n += rl;
    out[n++] = 0x02;
    out[n++] = (u8)sl;
    std::memcpy(out + n, sp, sl);
    n += sl;
    return n;
}

static Fe fe_from_scalar(const Scalar& a) {
    Fe f;
    std::memcpy(f.v, a.v, 32);  // a < n < p
    return f;
}

bool ecdsa_verify(const Scalar& r, const Scalar& s, const u8 msg32[32], const Ge& q) {
    if (r.is_zero() || s.is_zero() || q.inf) return false;
    const Scalar z = sc_from_be(msg32);
    const Scalar w = sc_inv(s);
    const Gej R = mul_double(sc_mul(r, w), q, sc_mul(z, w));
    if (R.inf) return false;
    // x(R) mod n == r  <=>  X == r' * Z^2 for r' in {r, r + n} (r + n < p)
    const Fe zz = fe_sqr(R.z);
    Fe rx = fe_from_scalar(r);
    if (fe_eq(fe_mul(rx, zz), R.x)) return true;
    const u64 pmn[4] = {0x402DA1722FC9BAEEULL, 0x4551231950B75FC4ULL, 1ULL, 0ULL};  // p - n
    if (geq(r.v, pmn)) return false;
    add4(rx.v, rx.v, kN);
    return fe_eq(fe_mul(rx, zz), R.x);
}

bool verify_der(const u8* pub, size_t publen, const u8* sig, size_t siglen, const u8 msg32[32]) {
    Ge q;
    if (!pubkey_parse(pub, publen, q)) return false;
    Scalar r, s;
    if (!sig_parse_der_lax(sig, siglen, r, s)) return false;
    if (sc_is_high(s)) s = sc_neg(s);  // CPubKey::Verify normalises to low S
    return ecdsa_verify(r, s, msg32, q);
}

namespace {

struct Rfc6979 {
    u8 K[32], V[32];
    bool retry = false;
    Rfc6979(const u8 key[32], const u8 msg[32], const u8* extra) {
        std::memset(V, 1, 32);
        std::memset(K, 0, 32);
        u8 buf[32 + 1 + 32 + 32 + 32];
        for (int round = 0; round < 2; ++round) {
            size_t n = 0;
            std::memcpy(buf, V, 32);
            n = 32;
            buf[n++] = (u8)round;
            std::memcpy(buf + n, key, 32);
            n += 32;
            std::memcpy(buf + n, msg, 32);
            n += 32;
            if (extra) {
                std::memcpy(buf + n, extra, 32);
                n += 32;
            }
            hmac_sha256(K, 32, buf, n, K);
            hmac_sha256(K, 32, V, 32, V);
        }
    }
    void next(u8 out[32]) {
        if (retry) {
            u8 buf[33];
            std::memcpy(buf, V, 32);
            buf[32] = 0;
            hmac_sha256(K, 32, buf, 33, K);
            hmac_sha256(K, 32, V, 32, V);
        }
        hmac_sha256(K, 32, V, 32, V);
        std::memcpy(out, V, 32);
        retry = true;
    }
};

}  // namespace

bool ecdsa_sign(const u8 msg32[32], const u8 key[32], Scalar& r, Scalar& s, int* recid, const u8* extra) {
    if (!seckey_valid(key)) return false;
    const Scalar d = sc_from_be(key), z = sc_from_be(msg32);
    Rfc6979 rng(key, msg32, extra);
    for (int attempt = 0; attempt < 1000; ++attempt) {
        u8 kb[32];
        rng.next(kb);
        bool of = false;
        const Scalar k = sc_from_be(kb, &of);
        if (of || k.is_zero()) continue;
        const Ge R = ge_from_gej(mul_gen(k));
        u8 xb[32];
        fe_to_be(R.x, xb);
        bool xof = false;
        r = sc_from_be(xb, &xof);
        if (r.is_zero()) continue;
        s = sc_mul(sc_inv(k), sc_add(z, sc_mul(r, d)));
        if (s.is_zero()) continue;
        int id = (fe_is_odd(R.y) ? 1 : 0) | (xof ? 2 : 0);
        if (sc_is_high(s)) {
            s = sc_neg(s);
            id ^= 1;
        }
        if (recid) *recid = id;
        return true;
    }
    return false;
}

bool sign_compact(const u8 msg32[32], const u8 key[32], bool compressed, u8 out[65]) {
    Scalar r, s;
    int recid = 0;
    if (!ecdsa_sign(msg32, key, r, s, &recid)) return false;
    out[0] = (u8)(27 + recid + (compressed ? 4 : 0));
    sc_to_be(r, out + 1);
    sc_to_be(s, out + 33);
    return true;
}

bool recover_compact(const u8 msg32[32], const u8 sig[65], Ge& out, bool& compressed) {
    const int h = sig[0] - 27;
    if (h < 0 || h > 7) return false;
    const int recid = h & 3;
    compressed = (h & 4) != 0;
    bool of1 = false, of2 = false;
    const Scalar r = sc_from_be(sig + 1, &of1), s = sc_from_be(sig + 33, &of2);
    if (of1 || of2 || r.is_zero() || s.is_zero()) return false;
    u8 xb[33];
    xb[0] = (recid & 1) ? 3 : 2;
    Fe x = fe_from_scalar(r);
    if (recid & 2) {
        const u64 pmn[4] = {0x402DA1722FC9BAEEULL, 0x4551231950B75FC4ULL, 1ULL, 0ULL};
        if (geq(r.v, pmn)) return false;
        add4(x.v, x.v, kN);
    }
    fe_to_be(x, xb + 1);
    Ge R;
    if (!pubkey_parse(xb, 33, R)) return false;
    const Scalar ri = sc_inv(r), z = sc_from_be(msg32);
    const Gej Q = mul_double(sc_mul(s, ri), R, sc_neg(sc_mul(z, ri)));
    if (Q.inf) return false;
    out = ge_from_gej(Q);
    return true;
}

bool seckey_tweak_add(u8 key[32], const u8 tweak[32]) {
    bool of = false;
    const Scalar t = sc_from_be(tweak, &of);
    if (of || !seckey_valid(key)) return false;
    const Scalar k = sc_add(sc_from_be(key), t);
    if (k.is_zero()) return false;
    sc_to_be(k, key);
    return true;
}

bool pubkey_tweak_add(Ge& p, const u8 tweak[32]) {
    bool of = false;
    const Scalar t = sc_from_be(tweak, &of);
    if (of || p.inf) return false;
    const Gej r = gej_add(gej_from_ge(p), mul_gen(t));
    if (r.inf) return false;
    p = ge_from_gej(r);
    return true;
}

}  // namespace nodexa::secp
