// Ethash building blocks: epoch seed, light cache, dataset items, epoch
// contexts, and classic hashimoto.
//
// Parity (behaviour, written from the Ethash spec):
//   sizes          src/crypto/ethash/lib/ethash/ethash.cpp:22-27, 365-393
//   largest prime  src/crypto/ethash/lib/ethash/primes.c:24-43
//   light cache    src/crypto/ethash/lib/ethash/ethash.cpp:101-129
//   dataset items  src/crypto/ethash/lib/ethash/ethash.cpp:180-251
//   epoch seed     src/crypto/ethash/lib/ethash/ethash.cpp:357-363
//   L1 cache       src/crypto/ethash/lib/ethash/ethash.cpp:168-170
//   managed ctx    src/crypto/ethash/lib/ethash/managed.cpp:84-100
// Differences by design: contexts are immutable and shared through a
// mutex-protected cache of shared_ptr (the reference's KAWPOWHash keeps an
// unlocked function-local static, src/hash.cpp:260-266 — a data race), and the
// optional host DAG is filled with per-item release/acquire publication.
#pragma once

#include <atomic>
#include <memory>
#include <mutex>
#include <string>

#include "../crypto/keccak.hpp"

namespace nodexa {

constexpr int kEpochLength = 7500;
constexpr int kLightCacheInitSize = 1 << 24;
constexpr int kLightCacheGrowth = 1 << 17;
constexpr int kLightCacheRounds = 3;
constexpr int kFullDatasetInitSize = 1 << 30;
constexpr int kFullDatasetGrowth = 1 << 23;
constexpr int kDatasetParents = 512;
constexpr int kEthashAccesses = 64;
constexpr int kL1CacheWords = 4096;  // 16 KiB KawPow L1

int find_largest_prime(int upper_bound);
int light_cache_num_items(int epoch);   // 512-bit items
int full_dataset_num_items(int epoch);  // 1024-bit items
inline int epoch_of_block(int block_number) { return block_number / kEpochLength; }
Hash256 epoch_seed(int epoch);
// Returns the epoch whose seed matches, or -1 (search bounded to 30000 epochs).
int find_epoch_number(const Hash256& seed);

struct EpochContext {
    int epoch = 0;
    int light_items = 0;
    int full_items = 0;  // 1024-bit items
    std::vector<Hash512> light;
    std::array<u32, kL1CacheWords> l1{};

    u64 light_bytes() const { return u64(light_items) * 64; }
    u64 full_bytes() const { return u64(full_items) * 128; }
};

void build_light_cache(Hash512* cache, int num_items, const Hash256& seed);
std::shared_ptr<const EpochContext> create_epoch_context(int epoch);
// Optional on-disk cache of light caches (empty dir = off). Loads verify a keccak256 checksum.
void set_light_cache_dir(const std::string& dir);
std::string light_cache_dir();
bool load_cached_light(EpochContext& ctx, const Hash256& seed);
void store_cached_light(const EpochContext& ctx, const Hash256& seed);
// Process-wide cache of recently used contexts (thread-safe, LRU of 4).
std::shared_ptr<const EpochContext> get_epoch_context(int epoch);

Hash512 dataset_item_512(const EpochContext& ctx, u64 index);
void dataset_item_1024(const EpochContext& ctx, u32 index, Hash512 out[2]);
void dataset_item_2048(const EpochContext& ctx, u32 index, Hash512 out[4]);

// Host-side full dataset, filled lazily (thread-safe) or eagerly in parallel.
class HostDag {
public:
    explicit HostDag(std::shared_ptr<const EpochContext> ctx);
    const EpochContext& ctx() const { return *ctx_; }
    // 2048-bit item i (= 512-bit items 4i..4i+3), computed on first use and
    // copied into `out`.
    void item2048(u32 index, Hash512 out[4]);
    void build_all(int threads);
    const Hash512* data() const { return items_.get(); }
    u64 num_items512() const { return n512_; }

private:
    std::shared_ptr<const EpochContext> ctx_;
    u64 n512_;
    std::unique_ptr<Hash512[]> items_;
    std::unique_ptr<std::atomic<u8>[]> ready_;  // per 2048-bit item
};

struct EthashResult {
    Hash256 final_hash;
    Hash256 mix_hash;
};
EthashResult ethash_hash(const EpochContext& ctx, const Hash256& header, u64 nonce);
bool ethash_verify(const EpochContext& ctx, const Hash256& header, const Hash256& mix, u64 nonce,
                   const Hash256& boundary);

}  // namespace nodexa
