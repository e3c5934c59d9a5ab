// Batch ECDSA verification on gfx950 (new; the reference verifies every signature serially on
// the CPU: CPubKey::Verify, src/pubkey.cpp:169, called from the script-check worker pool
// CCheckQueue, src/checkqueue.h:33-160, src/validation.cpp:9949). One thread per signature;
// arithmetic in secp256k1_device.hpp (host-testable, see csrc/crypto/secp256k1_model32.cpp).
//
// Per signature: public-key decompression (one sqrt chain), s^-1 mod n, u2*Q by a 2-bit window
// over affine {Q, 2Q, 3Q} (one batch inversion), u1*G by 64 mixed additions from a 64 KiB comb
// table that every thread reads (it stays in L1/L2), and the x(R) == r check in Jacobian
// coordinates. Work is the same for every lane (no data-dependent branches but the rare
// degenerate-addition flag), so waves do not diverge.
#include "kernel_params.h"
#include "secp256k1_device.hpp"

using namespace secp32;

extern "C" __global__ __launch_bounds__(256) void secp_verify_batch(SecpVerifyParams p) {
    const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
    if (idx >= p.n) return;
    const SecpVerifyJob& job = p.jobs[idx];
    const uint32_t kind = job.kind;
    uint32_t result = 0;
    if (kind == SECP_KIND_UNCOMPRESSED || kind == SECP_KIND_EVEN || kind == SECP_KIND_ODD) {
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
        bool ok;
        if (kind == SECP_KIND_UNCOMPRESSED) {
            ok = !f_geq_p(q.x) && !f_geq_p(q.y) && f_eq(f_sqr(q.y), rhs);
        } else {
            F y;
            ok = !f_geq_p(q.x) && f_sqrt(rhs, y);
            if ((y.v[0] & 1u) != (kind & 1u)) y = f_sub(f_zero(), y);
            q.y = y;
        }
        if (ok) result = (uint32_t)ecdsa_verify32(q, r, s, z, (const A*)p.gtab);
    }
    p.out[idx] = result;
}
