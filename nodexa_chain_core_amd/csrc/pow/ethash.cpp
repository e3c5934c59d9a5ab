#include "ethash.hpp"

#include <cstdio>
#include <list>
#include <mutex>
#include <string>
#include <thread>
#include <unistd.h>

namespace nodexa {

int find_largest_prime(int upper_bound) {
    int n = upper_bound;
    if (n < 2) return 0;
    if (n == 2) return 2;
    if ((n & 1) == 0) --n;
    for (;; n -= 2) {
        bool prime = true;
        for (int64_t d = 3; d * d <= n; d += 2)
            if (n % d == 0) { prime = false; break; }
        if (prime) return n;
    }
}

int light_cache_num_items(int epoch) {
    return find_largest_prime((kLightCacheInitSize + epoch * kLightCacheGrowth) / 64);
}

int full_dataset_num_items(int epoch) {
    return find_largest_prime(int((int64_t(kFullDatasetInitSize) + int64_t(epoch) * kFullDatasetGrowth) / 128));
}

Hash256 epoch_seed(int epoch) {
    Hash256 s;
    for (int i = 0; i < epoch; ++i) s = keccak256(s);
    return s;
}

int find_epoch_number(const Hash256& seed) {
    Hash256 s;
    for (int i = 0; i < 30000; ++i) {
        if (s == seed) return i;
        s = keccak256(s);
    }
    return -1;
}

void build_light_cache(Hash512* cache, int n, const Hash256& seed) {
    cache[0] = keccak512(seed.bytes, 32);
    for (int i = 1; i < n; ++i) cache[i] = keccak512(cache[i - 1]);
    for (int round = 0; round < kLightCacheRounds; ++round) {
        for (int i = 0; i < n; ++i) {
            const u32 v = cache[i].w32[0] % u32(n);
            const u32 w = u32((int64_t(n) + i - 1) % n);
            Hash512 x;
            for (int k = 0; k < 8; ++k) x.w64[k] = cache[v].w64[k] ^ cache[w].w64[k];
            cache[i] = keccak512(x);
        }
    }
}

namespace {

struct ItemState {
    const Hash512* cache;
    u64 n;
    u32 seed;
    Hash512 mix;

    ItemState(const EpochContext& ctx, u64 index)
        : cache(ctx.light.data()), n(u64(ctx.light_items)), seed(u32(index)) {
        mix = cache[index % n];
        mix.w32[0] ^= seed;
        mix = keccak512(mix);
    }
    inline void update(u32 round) {
        const u32 t = fnv1(seed ^ round, mix.w32[round % 16]);
        const Hash512& p = cache[t % n];
        for (int k = 0; k < 16; ++k) mix.w32[k] = fnv1(mix.w32[k], p.w32[k]);
    }
    Hash512 final() const { return keccak512(mix); }
};

}  // namespace

Hash512 dataset_item_512(const EpochContext& ctx, u64 index) {
    ItemState s(ctx, index);
    for (u32 j = 0; j < kDatasetParents; ++j) s.update(j);
    return s.final();
}

void dataset_item_1024(const EpochContext& ctx, u32 index, Hash512 out[2]) {
    ItemState a(ctx, u64(index) * 2), b(ctx, u64(index) * 2 + 1);
    for (u32 j = 0; j < kDatasetParents; ++j) { a.update(j); b.update(j); }
    out[0] = a.final();
    out[1] = b.final();
}

void dataset_item_2048(const EpochContext& ctx, u32 index, Hash512 out[4]) {
    ItemState a(ctx, u64(index) * 4), b(ctx, u64(index) * 4 + 1), c(ctx, u64(index) * 4 + 2),
        d(ctx, u64(index) * 4 + 3);
    for (u32 j = 0; j < kDatasetParents; ++j) { a.update(j); b.update(j); c.update(j); d.update(j); }
    out[0] = a.final();
    out[1] = b.final();
    out[2] = c.final();
    out[3] = d.final();
}

// ---------------------------------------------------------------- on-disk light-cache cache
// `-dagcache=<dir>` (SURVEY §5 checkpoint/resume): the serial light-cache build
// (2.3 s at epoch 384) is skipped on restart. File = 8-byte magic, the epoch
// seed, the item count, the payload and keccak256(payload); written to a temp
// file and renamed, so a crash never leaves a torn cache that would be trusted.
namespace {
std::mutex g_cache_mu;
std::string g_cache_dir;
constexpr char kCacheMagic[8] = {'N', 'X', 'L', 'I', 'G', 'H', 'T', '1'};

std::string cache_path(const EpochContext& ctx, const Hash256& seed) {
    return g_cache_dir + "/light-" + std::to_string(ctx.epoch) + "-" + hex_encode(seed.bytes, 8) + ".bin";
}
}  // namespace

void set_light_cache_dir(const std::string& dir) {
    std::lock_guard<std::mutex> g(g_cache_mu);
    g_cache_dir = dir;
}

std::string light_cache_dir() {
    std::lock_guard<std::mutex> g(g_cache_mu);
    return g_cache_dir;
}

bool load_cached_light(EpochContext& ctx, const Hash256& seed) {
    const std::string dir = light_cache_dir();
    if (dir.empty()) return false;
    FILE* f = std::fopen(cache_path(ctx, seed).c_str(), "rb");
    if (!f) return false;
    char magic[8];
    Hash256 fseed, sum;
    u32 items = 0;
    const size_t payload = ctx.light.size() * sizeof(Hash512);
    bool ok = std::fread(magic, 8, 1, f) == 1 && std::memcmp(magic, kCacheMagic, 8) == 0 &&
              std::fread(fseed.bytes, 32, 1, f) == 1 && std::memcmp(fseed.bytes, seed.bytes, 32) == 0 &&
              std::fread(&items, 4, 1, f) == 1 && int(items) == ctx.light_items &&
              std::fread(ctx.light.data(), payload, 1, f) == 1 && std::fread(sum.bytes, 32, 1, f) == 1;
    std::fclose(f);
    if (ok) ok = keccak256(reinterpret_cast<const u8*>(ctx.light.data()), payload) == sum;
    return ok;
}

void store_cached_light(const EpochContext& ctx, const Hash256& seed) {
    const std::string dir = light_cache_dir();
    if (dir.empty()) return;
    const std::string path = cache_path(ctx, seed);
    static std::atomic<u64> seq{0};  // unique per writer: several threads may store the same epoch
    const std::string tmp = path + ".tmp" + std::to_string(::getpid()) + "." + std::to_string(seq.fetch_add(1));
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return;
    const size_t payload = ctx.light.size() * sizeof(Hash512);
    const u32 items = u32(ctx.light_items);
    const Hash256 sum = keccak256(reinterpret_cast<const u8*>(ctx.light.data()), payload);
    bool ok = std::fwrite(kCacheMagic, 8, 1, f) == 1 && std::fwrite(seed.bytes, 32, 1, f) == 1 &&
              std::fwrite(&items, 4, 1, f) == 1 && std::fwrite(ctx.light.data(), payload, 1, f) == 1 &&
              std::fwrite(sum.bytes, 32, 1, f) == 1;
    ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) std::remove(tmp.c_str());
}

std::shared_ptr<const EpochContext> create_epoch_context(int epoch) {
    if (epoch < 0 || epoch > 30000) throw std::invalid_argument("epoch out of range");
    auto ctx = std::make_shared<EpochContext>();
    ctx->epoch = epoch;
    ctx->light_items = light_cache_num_items(epoch);
    ctx->full_items = full_dataset_num_items(epoch);
    ctx->light.resize(size_t(ctx->light_items));
    const Hash256 seed = epoch_seed(epoch);
    if (!load_cached_light(*ctx, seed)) {
        build_light_cache(ctx->light.data(), ctx->light_items, seed);
        store_cached_light(*ctx, seed);
    }
    // L1 = first 16 KiB of the dataset = 2048-bit items 0..63.
    Hash512 item[4];
    for (u32 i = 0; i < kL1CacheWords / 64; ++i) {
        dataset_item_2048(*ctx, i, item);
        std::memcpy(&ctx->l1[i * 64], item, 256);
    }
    return ctx;
}

std::shared_ptr<const EpochContext> get_epoch_context(int epoch) {
    static std::mutex mu;
    static std::list<std::shared_ptr<const EpochContext>> lru;
    {
        std::lock_guard<std::mutex> g(mu);
        for (auto it = lru.begin(); it != lru.end(); ++it)
            if ((*it)->epoch == epoch) {
                auto c = *it;
                lru.erase(it);
                lru.push_front(c);
                return c;
            }
    }
    auto ctx = create_epoch_context(epoch);  // built outside the lock
    std::lock_guard<std::mutex> g(mu);
    for (auto& c : lru)
        if (c->epoch == epoch) return c;
    lru.push_front(ctx);
    while (lru.size() > 4) lru.pop_back();
    return ctx;
}

HostDag::HostDag(std::shared_ptr<const EpochContext> ctx)
    : ctx_(std::move(ctx)), n512_(u64(ctx_->full_items) * 2) {
    items_.reset(new Hash512[n512_]);
    const u64 n2048 = u64(ctx_->full_items) / 2;
    ready_.reset(new std::atomic<u8>[n2048]);
    for (u64 i = 0; i < n2048; ++i) ready_[i].store(0, std::memory_order_relaxed);
}

void HostDag::item2048(u32 index, Hash512 out[4]) {
    std::atomic<u8>& flag = ready_[index];
    if (flag.load(std::memory_order_acquire) == 2) {
        std::memcpy(out, &items_[u64(index) * 4], 256);
        return;
    }
    dataset_item_2048(*ctx_, index, out);
    u8 expected = 0;
    if (flag.compare_exchange_strong(expected, 1, std::memory_order_acq_rel)) {
        std::memcpy(&items_[u64(index) * 4], out, 256);
        flag.store(2, std::memory_order_release);
    }
}

void HostDag::build_all(int threads) {
    if (threads <= 0) threads = int(std::max(1u, std::thread::hardware_concurrency()));
    std::atomic<u64> next{0};
    const u64 chunk = 4096;
    auto worker = [&] {
        for (;;) {
            const u64 lo = next.fetch_add(chunk);
            if (lo >= n512_) break;
            const u64 hi = std::min(n512_, lo + chunk);
            for (u64 i = lo; i < hi; ++i) items_[i] = dataset_item_512(*ctx_, i);
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) pool.emplace_back(worker);
    for (auto& t : pool) t.join();
    const u64 n2048 = u64(ctx_->full_items) / 2;
    for (u64 i = 0; i < n2048; ++i) ready_[i].store(2, std::memory_order_release);
}

// ---- classic Ethash hashimoto (src/crypto/ethash/lib/ethash/ethash.cpp:257-303, 416-440) ----
namespace {
Hash512 ethash_seed(const Hash256& header, u64 nonce) {
    u8 buf[40];
    std::memcpy(buf, header.bytes, 32);
    store_le64(buf + 32, nonce);
    return keccak512(buf, 40);
}
Hash256 ethash_final(const Hash512& seed, const Hash256& mix) {
    u8 buf[96];
    std::memcpy(buf, seed.bytes, 64);
    std::memcpy(buf + 64, mix.bytes, 32);
    return keccak256(buf, 96);
}
Hash256 ethash_mix(const EpochContext& ctx, const Hash512& seed) {
    u32 mix[32];
    for (int i = 0; i < 32; ++i) mix[i] = seed.w32[i % 16];
    const u32 seed0 = seed.w32[0];
    Hash512 item[2];
    for (u32 i = 0; i < kEthashAccesses; ++i) {
        const u32 p = fnv1(i ^ seed0, mix[i % 32]) % u32(ctx.full_items);
        dataset_item_1024(ctx, p, item);
        for (int j = 0; j < 16; ++j) mix[j] = fnv1(mix[j], item[0].w32[j]);
        for (int j = 0; j < 16; ++j) mix[16 + j] = fnv1(mix[16 + j], item[1].w32[j]);
    }
    Hash256 out;
    for (int i = 0; i < 32; i += 4) out.w32[i / 4] = fnv1(fnv1(fnv1(mix[i], mix[i + 1]), mix[i + 2]), mix[i + 3]);
    return out;
}
}  // namespace

EthashResult ethash_hash(const EpochContext& ctx, const Hash256& header, u64 nonce) {
    const Hash512 seed = ethash_seed(header, nonce);
    EthashResult r;
    r.mix_hash = ethash_mix(ctx, seed);
    r.final_hash = ethash_final(seed, r.mix_hash);
    return r;
}

bool ethash_verify(const EpochContext& ctx, const Hash256& header, const Hash256& mix, u64 nonce,
                   const Hash256& boundary) {
    const Hash512 seed = ethash_seed(header, nonce);
    if (!hash_le(ethash_final(seed, mix), boundary)) return false;
    return ethash_mix(ctx, seed) == mix;
}

}  // namespace nodexa
