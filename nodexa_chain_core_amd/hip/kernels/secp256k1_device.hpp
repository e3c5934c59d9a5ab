// secp256k1 arithmetic on 8 x 32-bit limbs for the gfx950 batch ECDSA verifier
// (secp256k1_verify.hip). The functions are host+device so the CPU test suite runs this exact
// code against the 64-bit golden model (csrc/crypto/secp256k1.cpp) — see
// csrc/crypto/secp256k1_model32.cpp.
//
// CDNA4 notes: every 32x32->64 product with a 64-bit addend is one v_mad_u64_u32, which issues
// at the full VALU rate on gfx950 (profiles/README r2b); a field multiplication is 64 of them plus
// the reduction by 2^256 = 2^32 + 977 (mod p). Points are Jacobian; the accumulator adds affine
// points only (mixed additions), and any addition that meets a doubling / inverse case sets
// `degenerate` so the host re-checks that signature on the CPU instead of trusting a special-
// case path that random signatures never exercise.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SECP_HD __host__ __device__ __forceinline__
#else
#define SECP_HD inline
#endif

namespace secp32 {

struct F {
    uint32_t v[8];
};

SECP_HD F f_zero() {
    F r;
    for (int i = 0; i < 8; ++i) r.v[i] = 0;
    return r;
}
SECP_HD F f_one() {
    F r = f_zero();
    r.v[0] = 1;
    return r;
}
SECP_HD bool f_is_zero(const F& a) {
    uint32_t x = 0;
    for (int i = 0; i < 8; ++i) x |= a.v[i];
    return x == 0;
}
SECP_HD bool f_eq(const F& a, const F& b) {
    uint32_t x = 0;
    for (int i = 0; i < 8; ++i) x |= a.v[i] ^ b.v[i];
    return x == 0;
}
SECP_HD F f_select(bool c, const F& a, const F& b) {  // c ? a : b
    F r;
    for (int i = 0; i < 8; ++i) r.v[i] = c ? a.v[i] : b.v[i];
    return r;
}

// ---------------------------------------------------------------- field mod p
// p = 2^256 - 2^32 - 977
SECP_HD bool f_geq_p(const F& a) {
    // p's limbs 2..7 are all ones: a >= p iff those are all ones and (a1, a0) >= (0xFFFFFFFE, 0xFFFFFC2F)
    uint32_t hi = 0xFFFFFFFFu;
    for (int i = 2; i < 8; ++i) hi &= a.v[i];
    if (hi != 0xFFFFFFFFu) return false;
    if (a.v[1] != 0xFFFFFFFEu) return a.v[1] > 0xFFFFFFFEu;
    return a.v[0] >= 0xFFFFFC2Fu;
}
// a + (2^32 + 977) * k for k < 2^34, returning the carry out of 2^256
SECP_HD uint32_t f_add_pc(F& a, uint64_t k) {
    uint64_t s = (uint64_t)a.v[0] + k * 977u;
    a.v[0] = (uint32_t)s;
    s = (s >> 32) + a.v[1] + k;
    a.v[1] = (uint32_t)s;
    uint32_t c = (uint32_t)(s >> 32);
    for (int i = 2; i < 8; ++i) {
        s = (uint64_t)a.v[i] + c;
        a.v[i] = (uint32_t)s;
        c = (uint32_t)(s >> 32);
    }
    return c;
}
SECP_HD F f_add(const F& a, const F& b) {
    F r;
    uint64_t c = 0;
    for (int i = 0; i < 8; ++i) {
        c += (uint64_t)a.v[i] + b.v[i];
        r.v[i] = (uint32_t)c;
        c >>= 32;
    }
    if (c || f_geq_p(r)) f_add_pc(r, 1);  // subtract p == add 2^256 - p modulo 2^256
    return r;
}
SECP_HD F f_sub(const F& a, const F& b) {
    F r;
    int64_t c = 0;
    for (int i = 0; i < 8; ++i) {
        c += (int64_t)a.v[i] - (int64_t)b.v[i];
        r.v[i] = (uint32_t)c;
        c >>= 32;  // arithmetic: 0 or -1
    }
    if (c) {  // borrow: add p = subtract (2^32 + 977) modulo 2^256
        int64_t d = (int64_t)r.v[0] - 977;
        r.v[0] = (uint32_t)d;
        d = (d >> 32) + (int64_t)r.v[1] - 1;
        r.v[1] = (uint32_t)d;
        d >>= 32;
        for (int i = 2; i < 8; ++i) {
            d += r.v[i];
            r.v[i] = (uint32_t)d;
            d >>= 32;
        }
    }
    return r;
}
SECP_HD F f_mul(const F& a, const F& b) {
    uint32_t t[16];
    for (int i = 0; i < 16; ++i) t[i] = 0;
    for (int i = 0; i < 8; ++i) {
        uint64_t c = 0;
        for (int j = 0; j < 8; ++j) {
            c += (uint64_t)a.v[i] * b.v[j] + t[i + j];
            t[i + j] = (uint32_t)c;
            c >>= 32;
        }
        t[i + 8] = (uint32_t)c;
    }
    // t_lo + t_hi * (2^32 + 977)
    F r;
    uint64_t c = 0;
    for (int k = 0; k < 8; ++k) {
        c += (uint64_t)t[8 + k] * 977u + t[k];
        if (k) c += t[7 + k];
        r.v[k] = (uint32_t)c;
        c >>= 32;
    }
    c += t[15];  // the top limb of t_hi << 32
    // fold the (< 2^34) overflow once more; a carry out of that is folded a last time
    const uint32_t k2 = f_add_pc(r, c);
    if (k2) f_add_pc(r, k2);
    if (f_geq_p(r)) f_add_pc(r, 1);
    return r;
}
SECP_HD F f_sqr(const F& a) { return f_mul(a, a); }
SECP_HD F f_sqr_n(F a, int n) {
#pragma unroll 1
    for (int i = 0; i < n; ++i) a = f_sqr(a);
    return a;
}
SECP_HD F f_mul_small(const F& a, uint32_t k) {
    F b = f_zero();
    b.v[0] = k;
    return f_mul(a, b);
}
// a^(2^223 - 1) and the small powers the sqrt / inverse chains reuse (libsecp256k1's chain)
struct PowChain {
    F x2, x3, x22, x223;
};
SECP_HD PowChain f_chain(const F& a) {
    PowChain c;
    c.x2 = f_mul(f_sqr(a), a);
    c.x3 = f_mul(f_sqr(c.x2), a);
    const F x6 = f_mul(f_sqr_n(c.x3, 3), c.x3);
    const F x9 = f_mul(f_sqr_n(x6, 3), c.x3);
    const F x11 = f_mul(f_sqr_n(x9, 2), c.x2);
    c.x22 = f_mul(f_sqr_n(x11, 11), x11);
    const F x44 = f_mul(f_sqr_n(c.x22, 22), c.x22);
    const F x88 = f_mul(f_sqr_n(x44, 44), x44);
    const F x176 = f_mul(f_sqr_n(x88, 88), x88);
    const F x220 = f_mul(f_sqr_n(x176, 44), x44);
    c.x223 = f_mul(f_sqr_n(x220, 3), c.x3);
    return c;
}
SECP_HD F f_inv(const F& a) {  // a^(p-2)
    const PowChain c = f_chain(a);
    F t = f_mul(f_sqr_n(c.x223, 23), c.x22);
    t = f_mul(f_sqr_n(t, 5), a);
    t = f_mul(f_sqr_n(t, 3), c.x2);
    return f_mul(f_sqr_n(t, 2), a);
}
SECP_HD bool f_sqrt(const F& a, F& r) {  // a^((p+1)/4), checked
    const PowChain c = f_chain(a);
    F t = f_mul(f_sqr_n(c.x223, 23), c.x22);
    t = f_mul(f_sqr_n(t, 6), c.x2);
    r = f_sqr_n(t, 2);
    return f_eq(f_sqr(r), a);
}

// ---------------------------------------------------------------- scalars mod n
// n = FFFFFFFF FFFFFFFF FFFFFFFF FFFFFFFE BAAEDCE6 AF48A03B BFD25E8C D0364141
SECP_HD bool s_geq_n(const F& a) {
    const uint32_t n[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                           0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    for (int i = 7; i >= 0; --i) {
        if (a.v[i] != n[i]) return a.v[i] > n[i];
    }
    return true;
}
// a + NC (2^256 - n) modulo 2^256, i.e. a - n when a >= n
SECP_HD void s_sub_n(F& a) {
    const uint32_t nc[5] = {0x2FC9BEBFu, 0x402DA173u, 0x50B75FC4u, 0x45512319u, 1u};
    uint64_t c = 0;
    for (int i = 0; i < 8; ++i) {
        c += (uint64_t)a.v[i] + (i < 5 ? nc[i] : 0u);
        a.v[i] = (uint32_t)c;
        c >>= 32;
    }
}
SECP_HD F s_mul(const F& a, const F& b) {
    const uint32_t nc[5] = {0x2FC9BEBFu, 0x402DA173u, 0x50B75FC4u, 0x45512319u, 1u};
    uint32_t t[16];
    for (int i = 0; i < 16; ++i) t[i] = 0;
    for (int i = 0; i < 8; ++i) {
        uint64_t c = 0;
        for (int j = 0; j < 8; ++j) {
            c += (uint64_t)a.v[i] * b.v[j] + t[i + j];
            t[i + j] = (uint32_t)c;
            c >>= 32;
        }
        t[i + 8] = (uint32_t)c;
    }
    // fold 1: t_lo + t_hi * NC  (< 2^386: 13 limbs)
    uint32_t u[13];
    for (int i = 0; i < 13; ++i) u[i] = i < 8 ? t[i] : 0u;
    for (int i = 0; i < 8; ++i) {
        uint64_t c = 0;
        for (int j = 0; j < 5; ++j) {
            c += (uint64_t)t[8 + i] * nc[j] + u[i + j];
            u[i + j] = (uint32_t)c;
            c >>= 32;
        }
        for (int k = i + 5; k < 13; ++k) {
            c += u[k];
            u[k] = (uint32_t)c;
            c >>= 32;
        }
    }
    // fold 2: u_lo + u_hi (5 limbs) * NC  (< 2^259: 9 limbs)
    uint32_t w[10];
    for (int i = 0; i < 10; ++i) w[i] = i < 8 ? u[i] : 0u;
    for (int i = 0; i < 5; ++i) {
        uint64_t c = 0;
        for (int j = 0; j < 5; ++j) {
            c += (uint64_t)u[8 + i] * nc[j] + w[i + j];
            w[i + j] = (uint32_t)c;
            c >>= 32;
        }
        for (int k = i + 5; k < 10; ++k) {
            c += w[k];
            w[k] = (uint32_t)c;
            c >>= 32;
        }
    }
    // fold 3: w_lo + (w8 + w9 * 2^32) * NC  (w8 < 8, w9 == 0): at most one carry past 2^256
    F r;
    uint64_t c = 0;
    for (int i = 0; i < 8; ++i) {
        c += (uint64_t)w[8] * (i < 5 ? nc[i] : 0u) + w[i];
        r.v[i] = (uint32_t)c;
        c >>= 32;
    }
    if (c) s_sub_n(r);  // value = r + 2^256 = r + NC (mod n)... r + NC cannot overflow again here
    if (s_geq_n(r)) s_sub_n(r);
    if (s_geq_n(r)) s_sub_n(r);
    return r;
}
SECP_HD F s_sqr_n(F a, int n) {
#pragma unroll 1
    for (int i = 0; i < n; ++i) a = s_mul(a, a);
    return a;
}
// a^(n-2) mod n: a^(2^127 - 1) by a chain, then the low 129 bits of n - 2 bit by bit
SECP_HD F s_inv(const F& a) {
    const F x2 = s_mul(s_mul(a, a), a);
    const F x3 = s_mul(s_mul(x2, x2), a);
    const F x6 = s_mul(s_sqr_n(x3, 3), x3);
    const F x12 = s_mul(s_sqr_n(x6, 6), x6);
    const F x24 = s_mul(s_sqr_n(x12, 12), x12);
    const F x48 = s_mul(s_sqr_n(x24, 24), x24);
    const F x96 = s_mul(s_sqr_n(x48, 48), x48);
    const F x120 = s_mul(s_sqr_n(x96, 24), x24);
    F t = s_mul(s_sqr_n(x120, 6), x6);  // 2^126 - 1
    t = s_mul(s_mul(t, t), a);          // 2^127 - 1
    // remaining exponent bits 128..0 of n - 2: bit 128 is 0, bits 127..0 = BAAEDCE6AF48A03BBFD25E8CD036413F
    const uint32_t low[4] = {0xD036413Fu, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u};
    t = s_mul(t, t);
#pragma unroll 1
    for (int i = 127; i >= 0; --i) {
        t = s_mul(t, t);
        const F ta = s_mul(t, a);
        const bool bit = (low[i >> 5] >> (i & 31)) & 1u;
        t = f_select(bit, ta, t);  // same work on every lane
    }
    return t;
}

// ---------------------------------------------------------------- points
struct J {  // Jacobian; inf flag carried separately
    F x, y, z;
};
struct A {  // affine
    F x, y;
};

// 2P (dbl-2009-l, a = 0); P must not be infinity (the caller tracks that)
SECP_HD J j_double(const J& p) {
    const F a = f_sqr(p.x), b = f_sqr(p.y), c = f_sqr(b);
    F d = f_sub(f_sub(f_sqr(f_add(p.x, b)), a), c);
    d = f_add(d, d);
    const F e = f_add(f_add(a, a), a), f = f_sqr(e);
    J r;
    r.x = f_sub(f, f_add(d, d));
    F c8 = f_add(c, c);
    c8 = f_add(c8, c8);
    c8 = f_add(c8, c8);
    r.y = f_sub(f_mul(e, f_sub(d, r.x)), c8);
    const F yz = f_mul(p.y, p.z);
    r.z = f_add(yz, yz);
    return r;
}
// P + Q with Q affine (madd-2007-bl). If P == +-Q the formula does not apply: `degenerate` is set.
SECP_HD J j_add_affine(const J& p, const A& q, bool& degenerate) {
    const F z1z1 = f_sqr(p.z);
    const F u2 = f_mul(q.x, z1z1), s2 = f_mul(f_mul(q.y, p.z), z1z1);
    const F h = f_sub(u2, p.x);
    F rr = f_sub(s2, p.y);
    if (f_is_zero(h)) degenerate = true;
    rr = f_add(rr, rr);
    const F hh = f_sqr(h);
    F i = f_add(hh, hh);
    i = f_add(i, i);
    const F j = f_mul(h, i), v = f_mul(p.x, i);
    J r;
    r.x = f_sub(f_sub(f_sqr(rr), j), f_add(v, v));
    const F yj = f_mul(p.y, j);
    r.y = f_sub(f_mul(rr, f_sub(v, r.x)), f_add(yj, yj));
    r.z = f_sub(f_sub(f_sqr(f_add(p.z, h)), z1z1), hh);
    return r;
}
SECP_HD J j_from_affine(const A& a) {
    J r;
    r.x = a.x;
    r.y = a.y;
    r.z = f_one();
    return r;
}
// acc (+)= q with an infinity flag on acc; `take` = false leaves acc unchanged (branch-free select)
SECP_HD void j_accumulate(J& acc, bool& acc_inf, const A& q, bool take, bool& degenerate) {
    bool deg = false;
    const J s = j_add_affine(acc, q, deg);
    const J qa = j_from_affine(q);
    const bool use_q = take && acc_inf;
    const bool use_s = take && !acc_inf;
    if (use_s && deg) degenerate = true;
    acc.x = f_select(use_q, qa.x, f_select(use_s, s.x, acc.x));
    acc.y = f_select(use_q, qa.y, f_select(use_s, s.y, acc.y));
    acc.z = f_select(use_q, qa.z, f_select(use_s, s.z, acc.z));
    acc_inf = acc_inf && !take;
}
SECP_HD A a_from_j(const J& p) {
    const F zi = f_inv(p.z), zi2 = f_sqr(zi);
    A r;
    r.x = f_mul(p.x, zi2);
    r.y = f_mul(p.y, f_mul(zi2, zi));
    return r;
}

// One signature: q affine (already on the curve), r and low-S s in [1, n), z = message mod n.
// gtab = 64 x 16 affine points j * 16^i * G (entry j = 0 unused). Returns 1 valid, 0 invalid,
// 2 "degenerate: recheck on the host".
SECP_HD int ecdsa_verify32(const A& q, const F& r, const F& s, const F& z, const A* gtab) {
    if (f_is_zero(r) || f_is_zero(s)) return 0;
    const F w = s_inv(s);
    const F u1 = s_mul(z, w), u2 = s_mul(r, w);
    bool degenerate = false;
    // 2-bit window over u2 with q, 2q, 3q in affine (one inversion converts the two)
    bool d0 = false;
    const J q2 = j_double(j_from_affine(q));
    const J q3 = j_add_affine(q2, q, d0);
    if (d0) degenerate = true;
    // batch-invert the two z's
    const F zz = f_mul(q2.z, q3.z), zzi = f_inv(zz);
    const F z2i = f_mul(zzi, q3.z), z3i = f_mul(zzi, q2.z);
    A t[3];
    t[0] = q;
    {
        const F a2 = f_sqr(z2i), b2 = f_sqr(z3i);
        t[1].x = f_mul(q2.x, a2);
        t[1].y = f_mul(q2.y, f_mul(a2, z2i));
        t[2].x = f_mul(q3.x, b2);
        t[2].y = f_mul(q3.y, f_mul(b2, z3i));
    }
    J acc;
    acc.x = acc.y = acc.z = f_one();
    bool inf = true;
#pragma unroll 1
    for (int i = 127; i >= 0; --i) {
        if (!inf) {
            acc = j_double(acc);
            acc = j_double(acc);
        }
        const uint32_t bits = (u2.v[i >> 4] >> ((i & 15) * 2)) & 3u;
        const A sel = {f_select(bits == 1, t[0].x, f_select(bits == 2, t[1].x, t[2].x)),
                       f_select(bits == 1, t[0].y, f_select(bits == 2, t[1].y, t[2].y))};
        j_accumulate(acc, inf, sel, bits != 0, degenerate);
    }
    // + u1 * G from the comb table: 64 nibbles, one mixed addition each
#pragma unroll 1
    for (int i = 0; i < 64; ++i) {
        const uint32_t nb = (u1.v[i >> 3] >> ((i & 7) * 4)) & 15u;
        const A g = gtab[i * 16 + (nb ? nb : 1)];
        j_accumulate(acc, inf, g, nb != 0, degenerate);
    }
    if (degenerate) return 2;
    if (inf) return 0;
    // x(R) mod n == r  <=>  X == r' Z^2 for r' in {r, r + n} (r + n < p)
    const F zz2 = f_sqr(acc.z);
    if (f_eq(f_mul(r, zz2), acc.x)) return 1;
    // p - n = 14551231950B75FC4402DA1722FC9BAEE
    const F pmn = {{0x2FC9BAEEu, 0x402DA172u, 0x50B75FC4u, 0x45512319u, 1u, 0u, 0u, 0u}};
    bool lt = false;
    for (int i = 7; i >= 0; --i) {
        if (r.v[i] != pmn.v[i]) {
            lt = r.v[i] < pmn.v[i];
            break;
        }
    }
    if (!lt) return 0;
    const uint32_t nl[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                            0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    F rn;
    uint64_t c = 0;
    for (int i = 0; i < 8; ++i) {
        c += (uint64_t)r.v[i] + nl[i];
        rn.v[i] = (uint32_t)c;
        c >>= 32;
    }
    return f_eq(f_mul(rn, zz2), acc.x) ? 1 : 0;
}

}  // namespace secp32
