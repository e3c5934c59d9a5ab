// Host build of the gfx950 ECDSA verifier's arithmetic (hip/kernels/secp256k1_device.hpp) plus
// the job packer shared with the GPU path: the CPU test suite checks the 32-bit-limb code
// against the 64-bit golden model (secp256k1.cpp) before any GPU run.
#include "secp256k1_model32.hpp"

#include <cstring>

#include "../../hip/kernels/secp256k1_device.hpp"
#include "secp256k1.hpp"

namespace nodexa::secp {

namespace {

void be32_to_limbs(const u8 b[32], uint32_t out[8]) {
    for (int i = 0; i < 8; ++i) {
        const u8* p = b + (7 - i) * 4;
        out[i] = (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
    }
}

}  // namespace

void pack_verify_job(const u8* pub, size_t publen, const u8* sig, size_t siglen, const u8 msg32[32],
                     SecpVerifyJob& job) {
    std::memset(&job, 0, sizeof(job));
    job.kind = SECP_KIND_INVALID;
    Scalar r, s;
    if (!sig_parse_der_lax(sig, siglen, r, s)) return;
    if (sc_is_high(s)) s = sc_neg(s);  // CPubKey::Verify normalises to low S
    u8 b[32];
    sc_to_be(r, b);
    be32_to_limbs(b, job.r);
    sc_to_be(s, b);
    be32_to_limbs(b, job.s);
    be32_to_limbs(msg32, job.z);
    if (publen == 33 && (pub[0] == 2 || pub[0] == 3)) {
        be32_to_limbs(pub + 1, job.x);
        job.kind = pub[0] == 2 ? SECP_KIND_EVEN : SECP_KIND_ODD;
    } else if (publen == 65 && (pub[0] == 4 || pub[0] == 6 || pub[0] == 7)) {
        // hybrid keys (06/07) carry y; their parity byte must match it
        if (pub[0] != 4 && (pub[64] & 1) != (pub[0] & 1)) return;
        be32_to_limbs(pub + 1, job.x);
        be32_to_limbs(pub + 33, job.y);
        job.kind = SECP_KIND_UNCOMPRESSED;
    }
}

void export_gen_table32(uint32_t* out) {
    // j * 16^i * G in affine, 16 limbs (x then y) per entry; entry j = 0 (infinity) is zero
    Gej base = gej_from_ge(generator());
    for (int i = 0; i < 64; ++i) {
        Gej acc;
        std::memset(out + (i * 16) * 16, 0, 64);
        for (int j = 1; j < 16; ++j) {
            acc = gej_add(acc, base);
            const Ge a = ge_from_gej(acc);
            u8 b[32];
            fe_to_be(a.x, b);
            be32_to_limbs(b, out + (i * 16 + j) * 16);
            fe_to_be(a.y, b);
            be32_to_limbs(b, out + (i * 16 + j) * 16 + 8);
        }
        for (int k = 0; k < 4; ++k) base = gej_double(base);
    }
}

const uint32_t* gen_table32() {
    static const std::vector<uint32_t> t = [] {
        std::vector<uint32_t> v(64 * 16 * 16);
        export_gen_table32(v.data());
        return v;
    }();
    return t.data();
}

int verify_job_model32(const SecpVerifyJob& job) {
    using namespace secp32;
    if (job.kind != SECP_KIND_UNCOMPRESSED && job.kind != SECP_KIND_EVEN && job.kind != SECP_KIND_ODD) return 0;
    A q;
    F r, s, z;
    for (int i = 0; i < 8; ++i) {
        q.x.v[i] = job.x[i];
        q.y.v[i] = job.y[i];
        r.v[i] = job.r[i];
        s.v[i] = job.s[i];
        z.v[i] = job.z[i];
    }
    if (s_geq_n(z)) s_sub_n(z);
    const F rhs = f_add(f_mul(f_sqr(q.x), q.x), f_mul_small(f_one(), 7));
    if (job.kind == SECP_KIND_UNCOMPRESSED) {
        if (f_geq_p(q.x) || f_geq_p(q.y) || !f_eq(f_sqr(q.y), rhs)) return 0;
    } else {
        F y;
        if (f_geq_p(q.x) || !f_sqrt(rhs, y)) return 0;
        if ((y.v[0] & 1u) != (job.kind & 1u)) y = f_sub(f_zero(), y);
        q.y = y;
    }
    return ecdsa_verify32(q, r, s, z, reinterpret_cast<const A*>(gen_table32()));
}

}  // namespace nodexa::secp
