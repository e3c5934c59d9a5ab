// Signature cache: see sigcache.hpp.
#include "sigcache.hpp"

#include <cstring>
#include <deque>
#include <mutex>
#include <random>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <utility>

#include "../crypto/sha256.hpp"

namespace nodexa {

namespace {

constexpr size_t kDefaultMaxBytes = size_t(32) << 20;  // DEFAULT_MAX_SIG_CACHE_SIZE (32 MiB)

struct KeyHash {
    size_t operator()(const std::string& k) const {
        size_t h;
        std::memcpy(&h, k.data(), sizeof(h));  // the key is already a salted SHA-256
        return h;
    }
};

}  // namespace

struct SigCache::Impl {
    mutable std::shared_mutex mu;
    // live entries with the insertion generation of their slot in `order`: an entry erased by
    // get(erase) and stored again later owns only its newest slot, so eviction of the stale slot
    // (a generation that no longer matches) leaves the re-inserted entry alone
    std::unordered_map<std::string, uint64_t, KeyHash> set;
    std::deque<std::pair<std::string, uint64_t>> order;  // insertion order, for eviction of the oldest
    uint64_t gen = 0;
    size_t max_entries = kDefaultMaxBytes / 32;
    u8 salt[32];
    uint64_t hits = 0, misses = 0, inserts = 0, evictions = 0;

    // drop the oldest slot; evicts its entry only if the slot is the entry's current one
    void pop_oldest() {
        auto& f = order.front();
        auto it = set.find(f.first);
        if (it != set.end() && it->second == f.second) {
            set.erase(it);
            ++evictions;
        }
        order.pop_front();
    }

    Impl() {
        std::random_device rd;
        for (auto& b : salt) b = u8(rd());
    }
    std::string key(const u8 msg[32], const Bytes& pubkey, const Bytes& sig) const {
        Bytes m;
        m.reserve(32 + 32 + pubkey.size() + sig.size());
        m.insert(m.end(), salt, salt + 32);
        m.insert(m.end(), msg, msg + 32);
        m.insert(m.end(), pubkey.begin(), pubkey.end());
        m.insert(m.end(), sig.begin(), sig.end());
        u8 out[32];
        sha256(m.data(), m.size(), out);
        return std::string(reinterpret_cast<const char*>(out), 32);
    }
};

SigCache::SigCache() : impl_(new Impl) {}

SigCache& SigCache::instance() {
    static SigCache cache;
    return cache;
}

void SigCache::set_max_bytes(size_t bytes) {
    std::unique_lock<std::shared_mutex> g(impl_->mu);
    impl_->max_entries = bytes / 32;
    while (impl_->set.size() > impl_->max_entries && !impl_->order.empty()) impl_->pop_oldest();
}

bool SigCache::get(const u8 msg[32], const Bytes& pubkey, const Bytes& sig, bool erase) {
    const std::string k = impl_->key(msg, pubkey, sig);
    if (erase) {
        std::unique_lock<std::shared_mutex> g(impl_->mu);
        const bool hit = impl_->set.erase(k) > 0;  // its slot in `order` is skipped at eviction
        hit ? ++impl_->hits : ++impl_->misses;
        return hit;
    }
    std::shared_lock<std::shared_mutex> g(impl_->mu);
    const bool hit = impl_->set.count(k) > 0;
    // counters are statistics only: benign races between readers
    hit ? __atomic_add_fetch(&impl_->hits, 1, __ATOMIC_RELAXED) : __atomic_add_fetch(&impl_->misses, 1, __ATOMIC_RELAXED);
    return hit;
}

void SigCache::put(const u8 msg[32], const Bytes& pubkey, const Bytes& sig) {
    std::string k = impl_->key(msg, pubkey, sig);
    std::unique_lock<std::shared_mutex> g(impl_->mu);
    if (impl_->max_entries == 0) return;
    const uint64_t g_new = ++impl_->gen;
    if (!impl_->set.emplace(k, g_new).second) return;
    impl_->order.emplace_back(std::move(k), g_new);
    ++impl_->inserts;
    while (impl_->set.size() > impl_->max_entries && !impl_->order.empty()) impl_->pop_oldest();
    if (impl_->order.size() > 2 * impl_->max_entries + 1024) {  // drop the slots of erased entries
        std::deque<std::pair<std::string, uint64_t>> live;
        for (auto& x : impl_->order) {
            auto it = impl_->set.find(x.first);
            if (it != impl_->set.end() && it->second == x.second) live.push_back(x);
        }
        impl_->order.swap(live);
    }
}

void SigCache::clear() {
    std::unique_lock<std::shared_mutex> g(impl_->mu);
    impl_->set.clear();
    impl_->order.clear();
}

SigCache::Stats SigCache::stats() const {
    std::shared_lock<std::shared_mutex> g(impl_->mu);
    Stats s;
    s.entries = impl_->set.size();
    s.max_entries = impl_->max_entries;
    s.hits = impl_->hits;
    s.misses = impl_->misses;
    s.inserts = impl_->inserts;
    s.evictions = impl_->evictions;
    return s;
}

}  // namespace nodexa
