// secp256k1: field / scalar / group arithmetic, ECDSA verify and RFC 6979 signing,
// public-key parsing, lax DER parsing and compact recoverable signatures — written from the SEC 2
// curve definition for this engine (the reference vendors libsecp256k1, src/secp256k1/, and
// reaches it through CPubKey::Verify (src/pubkey.cpp:169-184, lax DER + low-S normalisation) and
// CKey::Sign / SignCompact (src/key.cpp)).
//
// Host code, not constant time for verification (public data only). Signing uses a fixed
// comb over a precomputed table of G; it is used for wallet / test keys, not for HSM-grade keys.
// The GPU batch verifier (hip/kernels/secp256k1_verify.hip) implements the same arithmetic on
// 32-bit limbs; this file is its golden model.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace nodexa::secp {

using u8 = uint8_t;
using u64 = uint64_t;

// Field element mod p = 2^256 - 2^32 - 977, 4 little-endian 64-bit limbs, always fully reduced.
struct Fe {
    u64 v[4] = {0, 0, 0, 0};
};
// Scalar mod n (the group order), fully reduced.
struct Scalar {
    u64 v[4] = {0, 0, 0, 0};
    bool is_zero() const { return (v[0] | v[1] | v[2] | v[3]) == 0; }
};
// Affine point (inf = point at infinity) and Jacobian point (x = X/Z^2, y = Y/Z^3).
struct Ge {
    Fe x, y;
    bool inf = true;
};
struct Gej {
    Fe x, y, z;
    bool inf = true;
};

// ---- field
Fe fe_from_be(const u8 b[32], bool* overflow = nullptr);  // reduced mod p
void fe_to_be(const Fe& a, u8 out[32]);
Fe fe_add(const Fe& a, const Fe& b);
Fe fe_sub(const Fe& a, const Fe& b);
Fe fe_neg(const Fe& a);
Fe fe_mul(const Fe& a, const Fe& b);
Fe fe_sqr(const Fe& a);
Fe fe_inv(const Fe& a);                  // a^(p-2); inv(0) = 0
bool fe_sqrt(const Fe& a, Fe& r);        // r^2 == a, false if a is a non-residue
bool fe_eq(const Fe& a, const Fe& b);
bool fe_is_zero(const Fe& a);
bool fe_is_odd(const Fe& a);

// ---- scalar
Scalar sc_from_be(const u8 b[32], bool* overflow = nullptr);  // reduced mod n
void sc_to_be(const Scalar& a, u8 out[32]);
Scalar sc_add(const Scalar& a, const Scalar& b);
Scalar sc_neg(const Scalar& a);
Scalar sc_mul(const Scalar& a, const Scalar& b);
Scalar sc_inv(const Scalar& a);
bool sc_is_high(const Scalar& a);  // a > n/2

// ---- group
const Ge& generator();
Gej gej_from_ge(const Ge& a);
Ge ge_from_gej(const Gej& a);
Gej gej_double(const Gej& a);
Gej gej_add(const Gej& a, const Gej& b);
Gej gej_add_ge(const Gej& a, const Ge& b);
bool ge_on_curve(const Ge& a);
Gej mul_gen(const Scalar& k);                                  // k*G (precomputed comb)
Gej mul(const Ge& p, const Scalar& k);                         // k*P
Gej mul_double(const Scalar& a, const Ge& p, const Scalar& b); // a*P + b*G

// ---- keys and signatures (Bitcoin encodings)
// 33-byte compressed (02/03), 65-byte uncompressed (04) or hybrid (06/07, parity checked).
bool pubkey_parse(const u8* in, size_t len, Ge& out);
size_t pubkey_serialize(const Ge& p, bool compressed, u8 out[65]);
bool seckey_valid(const u8 key[32]);
bool pubkey_create(const u8 key[32], Ge& out);

// libsecp256k1-compatible lax DER parse (src/pubkey.cpp ecdsa_signature_parse_der_lax): false only
// on a structural error; r or s that overflow give (0, 0), which never verifies.
bool sig_parse_der_lax(const u8* in, size_t len, Scalar& r, Scalar& s);
size_t sig_serialize_der(const Scalar& r, const Scalar& s, u8 out[72]);
// ECDSA verification of (r, s) over msg32 (s of either sign: the caller normalises as the
// reference does, i.e. high-S signatures verify).
bool ecdsa_verify(const Scalar& r, const Scalar& s, const u8 msg32[32], const Ge& q);
// DER signature -> verify, with CPubKey::Verify's semantics (lax DER, normalised S).
bool verify_der(const u8* pub, size_t publen, const u8* sig, size_t siglen, const u8 msg32[32]);
// RFC 6979 deterministic signing (HMAC-SHA256), low-S; `extra` optional 32-byte entropy.
// Returns false for an invalid key. recid receives the public-key recovery id (0..3).
bool ecdsa_sign(const u8 msg32[32], const u8 key[32], Scalar& r, Scalar& s, int* recid = nullptr,
                const u8* extra = nullptr);
// 65-byte compact signature (header 27 + recid + 4 if compressed) as CKey::SignCompact.
bool sign_compact(const u8 msg32[32], const u8 key[32], bool compressed, u8 out[65]);
// Recover the public key of a compact signature (CPubKey::RecoverCompact).
bool recover_compact(const u8 msg32[32], const u8 sig[65], Ge& out, bool& compressed);

// BIP32 helpers: key + tweak mod n (false if the result is invalid) and P + tweak*G.
bool seckey_tweak_add(u8 key[32], const u8 tweak[32]);
bool pubkey_tweak_add(Ge& p, const u8 tweak[32]);

}  // namespace nodexa::secp
