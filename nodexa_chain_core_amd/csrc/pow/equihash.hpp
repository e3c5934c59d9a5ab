// Equihash(n, k) — generalized birthday problem PoW (Biryukov & Khovratovich),
// instantiated as Zcash's Equihash(200, 9). NOT present in the reference
// (README.md:7 only claims it): built from the public
// Zcash protocol spec §7.6.1 for the engine's new, opt-in header extension.
//
//   X_i   = BLAKE2b-(512/n*n/8 bytes, personal "ZcashPoW"||le32(n)||le32(k))
//           (I || le32(i / (512/n)))[ (i % (512/n)) * n/8 : +n/8 ]
//   N     = 2^(n/(k+1)+1) leaves; a solution is 2^k distinct indices such that
//           the XOR of their X is 0, every subtree of size 2^l collides on its
//           first l*n/(k+1) bits, and every node's left subtree starts with the
//           smaller index. Indices are packed as (n/(k+1)+1)-bit big-endian
//           fields (1344 bytes for 200,9).
//
// This file is the CPU golden model (row generation, Wagner solver, verifier);
// the gfx950 solver lives in hip/kernels/equihash.hip.
#pragma once

#include <memory>

#include "../crypto/blake2b.hpp"

namespace nodexa {

struct EquihashParams {
    int n = 200;
    int k = 9;
    int collision_bits() const { return n / (k + 1); }
    int indices_per_hash() const { return 512 / n; }
    int hash_bytes() const { return n / 8; }
    int digest_bytes() const { return indices_per_hash() * n / 8; }
    u32 num_leaves() const { return 1u << (collision_bits() + 1); }
    int solution_indices() const { return 1 << k; }
    int solution_bytes() const { return solution_indices() * (collision_bits() + 1) / 8; }
    void personal(u8 out[16]) const;
};

// BLAKE2b state after absorbing the input I (shared by all rows of a nonce).
Blake2b equihash_base_state(const EquihashParams& p, const u8* input, size_t n);
// The n-bit string X_i (n/8 bytes, big-endian bit order).
void equihash_leaf(const EquihashParams& p, const Blake2b& base, u32 i, u8* out);

Bytes equihash_pack_indices(const EquihashParams& p, const std::vector<u32>& idx);
std::vector<u32> equihash_unpack_indices(const EquihashParams& p, const Bytes& sol);

// Verifier; `reason` gets the failing rule ("bad-size", "collision", "order", "duplicate", "nonzero").
bool equihash_verify(const EquihashParams& p, const u8* input, size_t n, const std::vector<u32>& indices,
                     std::string* reason = nullptr);

struct EquihashSolveStats {
    std::vector<u64> rows_per_round;
    u64 candidates = 0;
    u64 discarded_duplicates = 0;
};
// Wagner solver; returns canonical index lists (each verified).
std::vector<std::vector<u32>> equihash_solve_cpu(const EquihashParams& p, const u8* input, size_t n,
                                                 size_t max_solutions = 64, EquihashSolveStats* stats = nullptr,
                                                 int threads = 0);

}  // namespace nodexa

namespace pybind11 { class module_; }
void bind_equihash_cpu(pybind11::module_& m);
