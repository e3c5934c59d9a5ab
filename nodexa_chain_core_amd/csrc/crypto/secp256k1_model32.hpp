// Packing of ECDSA verification jobs for the gfx950 batch verifier and the host run of its
// 32-bit-limb arithmetic (see secp256k1_model32.cpp).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "../../hip/kernels/kernel_params.h"

namespace nodexa::secp {

// One job from a public key (any CPubKey encoding), a DER signature (hash type stripped) and the
// 32-byte message. Unparseable inputs give kind SECP_KIND_INVALID (result 0 on the device).
void pack_verify_job(const uint8_t* pub, size_t publen, const uint8_t* sig, size_t siglen, const uint8_t msg32[32],
                     SecpVerifyJob& job);
// The device's comb table of G: 64 x 16 affine points, 16 little-endian limbs each.
void export_gen_table32(uint32_t* out);
const uint32_t* gen_table32();
// The device code run on the host: 1 valid, 0 invalid, 2 degenerate (re-check with verify_der).
int verify_job_model32(const SecpVerifyJob& job);

}  // namespace nodexa::secp
