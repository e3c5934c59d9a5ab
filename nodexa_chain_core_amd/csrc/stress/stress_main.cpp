// Concurrency stress for the native core, built under ThreadSanitizer and
// AddressSanitizer+UBSan (SURVEY §5 "race detection": the reference's
// DEBUG_LOCKORDER / thread-safety annotations, plus the real race it has in
// KAWPOWHash's unlocked static epoch context, src/hash.cpp:260-266).
//
// Exercised concurrently: the shared epoch-context cache (get_epoch_context),
// the on-disk light-cache cache (same epoch stored by several threads), the
// lazily filled HostDag, light-mode KawPow hashing, the multi-threaded X16R
// nonce search, and HeaderChain with one writer and several readers.
// Exit status 0 = every cross-thread result agreed and no sanitizer report.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../chain/headerchain.hpp"
#include "../chain/params.hpp"
#include "../pow/ethash.hpp"
#include "../pow/kawpow.hpp"
#include "../pow/x16r.hpp"

using namespace nodexa;

static std::atomic<int> g_fail{0};
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            g_fail.fetch_add(1);                                          \
        }                                                                 \
    } while (0)

static void stress_epoch_and_kawpow(int epochs) {
    std::vector<std::thread> ts;
    std::vector<Hash256> out(8);
    for (int t = 0; t < 8; ++t)
        ts.emplace_back([t, epochs, &out] {
            const int e = t % epochs;  // threads race on the same cache entries
            auto ctx = get_epoch_context(e);
            Hash256 hh;
            hh.bytes[0] = 7;
            out[t] = kawpow_hash(*ctx, e * 7500 + 5, hh, 42).final_hash;
        });
    for (auto& th : ts) th.join();
    for (int t = epochs; t < 8; ++t) CHECK(out[t] == out[t % epochs]);
}

static void stress_light_cache_dir(const std::string& dir, int writers) {
    set_light_cache_dir(dir);
    std::vector<std::thread> ts;
    std::vector<std::shared_ptr<const EpochContext>> ctx(static_cast<size_t>(writers));
    for (int t = 0; t < writers; ++t) ts.emplace_back([t, &ctx] { ctx[size_t(t)] = create_epoch_context(0); });
    for (auto& th : ts) th.join();
    auto again = create_epoch_context(0);  // must load a complete, checksummed file
    for (int t = 0; t < writers; ++t) CHECK(ctx[size_t(t)]->light == again->light);
    set_light_cache_dir("");
}

static void stress_hostdag() {
    auto ctx = get_epoch_context(0);
    HostDag dag(ctx);
    std::vector<std::thread> ts;
    for (int t = 0; t < 6; ++t)
        ts.emplace_back([&dag, &ctx, t] {
            Hash512 got[4], want[4];
            for (u32 i = 0; i < 48; ++i) {
                const u32 idx = (i * 7 + u32(t)) % 64;  // heavy overlap between threads
                dag.item2048(idx, got);
                dataset_item_2048(*ctx, idx, want);
                for (int k = 0; k < 4; ++k) CHECK(got[k] == want[k]);
            }
        });
    for (auto& th : ts) th.join();
}

static void stress_x16r() {
    u8 hdr[80] = {0};
    for (int i = 0; i < 80; ++i) hdr[i] = u8(i * 3 + 1);
    u8 target[32];
    for (auto& b : target) b = 0xff;
    target[31] = 0x0f;  // ~1/16 of hashes qualify
    std::vector<std::thread> ts;
    std::vector<X16rSearchResult> r(2);
    for (int t = 0; t < 2; ++t) ts.emplace_back([&, t] { r[t] = x16r_search(hdr, true, target, 0, 256, 4); });
    for (auto& th : ts) th.join();
    CHECK(r[0].found && r[1].found && r[0].nonce == r[1].nonce);
}

static void stress_headerchain() {
    ChainParams p = make_chain_params("regtest");
    p.kawpow_activation_time = p.genesis.header.time;
    HeaderChain chain(p, std::make_shared<CpuPowVerifier>());
    std::atomic<bool> done{false};
    std::vector<std::thread> readers;
    for (int t = 0; t < 3; ++t)
        readers.emplace_back([&] {
            while (!done.load()) {
                const HeaderIndex* tip = chain.tip();
                CHECK(tip != nullptr);
                const int h = chain.height();
                CHECK(chain.at_height(h / 2) != nullptr);
                CHECK(chain.find(tip->hash) != nullptr);
            }
        });
    const HeaderIndex* prev = chain.tip();
    u32 t = p.genesis.header.time;
    for (int h = 1; h <= 400; ++h) {
        BlockHeader b;
        b.version = 0x30000000;
        b.prev = prev->hash;
        b.merkle_root.data[0] = u8(h);
        b.merkle_root.data[1] = u8(h >> 8);
        t += 61;
        b.time = t;
        b.height = u32(h);
        b.bits = chain.next_bits(b);
        AcceptResult r = chain.accept_header(b, t + 10, false);
        CHECK(r.ok);
        if (!r.ok) break;
        prev = r.index;
    }
    done = true;
    for (auto& th : readers) th.join();
    CHECK(chain.height() == 400);
}

// accept_headers' linear-batch path on a DGW network: contextual rules on the pool, a run on top
// of the tip built on the pool (entries constructed and inserted into the block-index table
// concurrently), then header-by-header for the part that forks.
static void stress_headerchain_batch() {
    ChainParams p = make_chain_params("test");
    p.kawpow_activation_time = p.genesis.header.time;
    auto verifier = std::make_shared<CpuPowVerifier>();
    HeaderChain scratch(p, verifier);
    std::vector<BlockHeader> hs;
    const HeaderIndex* prev = scratch.tip();
    u32 t = p.genesis.header.time;
    for (int h = 1; h <= 1500; ++h) {
        BlockHeader b;
        b.version = 0x30000000;
        b.prev = prev->hash;
        b.merkle_root.data[0] = u8(h);
        b.merkle_root.data[1] = u8(h >> 8);
        t += 50 + (h * 7) % 40;
        b.time = t;
        b.height = u32(h);
        b.bits = scratch.next_bits(b);
        AcceptResult r = scratch.accept_header(b, t + 10, false);
        CHECK(r.ok);
        if (!r.ok) return;
        prev = r.index;
        hs.push_back(b);
    }
    for (int round = 0; round < 3; ++round) {
        HeaderChain chain(p, verifier);
        const auto r = chain.accept_headers(hs.data(), hs.size(), int64_t(t) + 10, false, nullptr, nullptr);
        CHECK(r.size() == hs.size() && r.back().ok);
        CHECK(chain.height() == 1500 && chain.tip()->hash == scratch.tip()->hash);
        CHECK(chain.tip()->chain_work == scratch.tip()->chain_work);
        for (int h = 0; h <= 1500; h += 37) CHECK(chain.tip()->ancestor(h) == chain.at_height(h));
    }
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    const bool quick = argc > 2 && std::string(argv[2]) == "--quick";  // one epoch (CI)
    stress_epoch_and_kawpow(quick ? 1 : 2);
    stress_light_cache_dir(dir, quick ? 2 : 4);
    stress_hostdag();
    stress_x16r();
    stress_headerchain();
    stress_headerchain_batch();
    std::printf("stress: %s (%d failed checks)\n", g_fail.load() ? "FAIL" : "ok", g_fail.load());
    return g_fail.load() ? 1 : 0;
}
