// Signature cache: CSignatureCache (src/script/sigcache.cpp:76-86) — the ECDSA checks a transaction
// passed when it entered the mempool are remembered, so connecting the block that confirms it does
// not verify them again (on the host or in the GPU batch).
//
// Entries are SHA256(salt || message hash || pubkey || signature) with a per-process random salt
// (an attacker cannot aim collisions at the table). The table is bounded (-maxsigcachesize, bytes
// of 32-byte entries) and evicts the oldest entries first. Like the reference, a lookup made while
// validating a block erases the entry it hits (the transaction is then confirmed: its signatures
// will not be asked for again), while mempool acceptance inserts.
#pragma once
#include <cstddef>
#include <cstdint>

#include "../util/common.hpp"

namespace nodexa {

class SigCache {
public:
    static SigCache& instance();
    void set_max_bytes(size_t bytes);
    bool get(const u8 msg[32], const Bytes& pubkey, const Bytes& sig, bool erase);
    void put(const u8 msg[32], const Bytes& pubkey, const Bytes& sig);
    void clear();
    struct Stats {
        size_t entries = 0, max_entries = 0;
        uint64_t hits = 0, misses = 0, inserts = 0, evictions = 0;
    };
    Stats stats() const;

private:
    SigCache();
    struct Impl;
    Impl* impl_;
};

}  // namespace nodexa
