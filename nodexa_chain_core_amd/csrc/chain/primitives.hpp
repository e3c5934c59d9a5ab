// Transactions, block headers (80/120 B), blocks and merkle roots.
//
// Parity: CTransaction / CMutableTransaction segwit serialization
// (src/primitives/transaction.h:184-272,391), CBlockHeader / CBlock
// (src/primitives/block.h:38-177), CKAWPOWInput (:213-233), GetHash /
// GetHashFull / GetKAWPOWHeaderHash dispatch (src/primitives/block.cpp:38-99),
// ComputeMerkleRoot / BlockMerkleRoot / BlockWitnessMerkleRoot
// (src/consensus/merkle.cpp:136-180).
//
// Unlike the reference, the KawPow activation time is not a process global
// (nKAWPOWActivationTime): it is an explicit parameter, so one process can hold
// headers of several networks (and tests can switch regtest to KawPow).
#pragma once

#include <memory>

#include "serialize.hpp"
#include "uint256.hpp"

namespace nodexa {

using Amount = int64_t;
constexpr Amount COIN = 100000000;

struct OutPoint {
    Uint256 hash;
    u32 n = 0xffffffffu;
    bool is_null() const { return hash.is_null() && n == 0xffffffffu; }
};

struct TxIn {
    OutPoint prevout;
    Bytes script_sig;
    u32 sequence = 0xffffffffu;
    std::vector<Bytes> witness;
};

struct TxOut {
    Amount value = -1;
    Bytes script_pubkey;
};

struct Transaction {
    int32_t version = 1;
    std::vector<TxIn> vin;
    std::vector<TxOut> vout;
    u32 lock_time = 0;

    bool has_witness() const {
        for (auto& i : vin) if (!i.witness.empty()) return true;
        return false;
    }
    bool is_coinbase() const { return vin.size() == 1 && vin[0].prevout.is_null(); }
    void serialize(Writer& w, bool with_witness = true) const;
    static Transaction deserialize(Reader& r, bool allow_witness = true);
    Bytes bytes(bool with_witness = true) const { Writer w; serialize(w, with_witness); return w.buf; }
    Uint256 txid() const;   // sha256d of the non-witness serialization
    Uint256 wtxid() const;  // sha256d of the full serialization
    Amount value_out() const { Amount s = 0; for (auto& o : vout) s += o.value; return s; }
};

enum class PowAlgo { X16R, X16RV2, KAWPOW };

// Equihash(200,9) header extension (new). The
// reference has no Equihash, so the extension must leave every reference
// header byte-identical: it is flagged by a version bit no reference network
// sets, and consensus only allows it from ChainParams::equihash_activation_time
// (never set on main/test/regtest by default). An extended header is
//   version|prev|merkle|time|bits|height | nonce256 | CompactSize(1344) solution
// i.e. the KawPow 80-byte CKAWPOWInput prefix followed by a 32-byte nonce and
// the 512 x 21-bit packed index solution; the Equihash input is those
// 80 + 32 bytes, and the block hash (the PoW hash compared to nBits) is the
// SHA256d of the whole serialized header, as in Zcash.
constexpr int32_t kEquihashVersionBit = 1 << 26;

struct BlockHeader {
    int32_t version = 0;
    Uint256 prev;
    Uint256 merkle_root;
    u32 time = 0;
    u32 bits = 0;
    u32 nonce = 0;
    // KawPow fields (serialized iff time >= kawpow_activation_time)
    u32 height = 0;
    u64 nonce64 = 0;
    Uint256 mix_hash;
    // Equihash extension fields (serialized iff version & kEquihashVersionBit)
    Uint256 nonce256;
    Bytes solution;

    bool is_kawpow(u32 kawpow_activation_time) const { return time >= kawpow_activation_time; }
    bool is_equihash() const { return (version & kEquihashVersionBit) != 0; }
    Bytes equihash_input() const;  // kawpow_input() || nonce256 (112 bytes)
    Uint256 equihash_hash(u32 kawpow_activation_time) const;  // SHA256d(serialized header)
    void serialize(Writer& w, u32 kawpow_activation_time) const;
    static BlockHeader deserialize(Reader& r, u32 kawpow_activation_time);
    Bytes bytes(u32 kawpow_activation_time) const { Writer w; serialize(w, kawpow_activation_time); return w.buf; }
    Bytes legacy80() const;      // nVersion..nNonce (X16R input)
    Bytes kawpow_input() const;  // 80-byte CKAWPOWInput
    Uint256 kawpow_header_hash() const;  // SerializeHash(CKAWPOWInput)
};

struct Block {
    BlockHeader header;
    std::vector<Transaction> vtx;
    void serialize(Writer& w, u32 kawpow_activation_time, bool with_witness = true) const;
    static Block deserialize(Reader& r, u32 kawpow_activation_time);
    Bytes bytes(u32 kawpow_activation_time, bool with_witness = true) const {
        Writer w;
        serialize(w, kawpow_activation_time, with_witness);
        return w.buf;
    }
    size_t stripped_size(u32 act) const { return bytes(act, false).size(); }
    size_t total_size(u32 act) const { return bytes(act, true).size(); }
    size_t weight(u32 act) const { return stripped_size(act) * 3 + total_size(act); }
};

Uint256 compute_merkle_root(std::vector<Uint256> leaves, bool* mutated = nullptr);
Uint256 block_merkle_root(const Block& b, bool* mutated = nullptr);
Uint256 block_witness_merkle_root(const Block& b, bool* mutated = nullptr);
// Index of the witness commitment output in the coinbase, or -1 (GetWitnessCommitmentIndex).
int witness_commitment_index(const Block& b);

}  // namespace nodexa
