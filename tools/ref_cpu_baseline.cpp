// Reference CPU KawPow baseline harness (BASELINE.md "How the reference number
// will be established"). Links the reference's own ethash/ProgPoW sources
// (compiled from /root/reference/src/crypto/ethash, nothing of it is copied
// here) and times progpow::search — the function the reference's miner calls
// (src/miner.cpp:728-759 -> src/crypto/ethash/lib/ethash/progpow.cpp:567-579)
// — over the full, pre-filled epoch dataset on all host cores.
//
//   tools/ref_cpu_baseline.sh [epoch] [seconds]
#include <crypto/ethash/include/ethash/progpow.hpp>
#include <crypto/ethash/lib/ethash/ethash-internal.hpp>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

int main(int argc, char** argv) {
    const int epoch = argc > 1 ? std::atoi(argv[1]) : 384;
    const double seconds = argc > 2 ? std::atof(argv[2]) : 20.0;
    const unsigned threads = std::thread::hardware_concurrency();
    const int block = epoch * 7500 + 123;
    using clk = std::chrono::steady_clock;

    auto t0 = clk::now();
    ethash_epoch_context_full* ctx = ethash_create_epoch_context_full(epoch);
    if (!ctx) { std::fprintf(stderr, "context allocation failed\n"); return 1; }
    const uint32_t n1024 = (uint32_t)ctx->full_dataset_num_items;
    std::atomic<uint32_t> next{0};
    auto fill = [&] {
        for (;;) {
            const uint32_t b = next.fetch_add(4096);
            if (b >= n1024) return;
            const uint32_t e = b + 4096 < n1024 ? b + 4096 : n1024;
            for (uint32_t i = b; i < e; ++i) ctx->full_dataset[i] = ethash::calculate_dataset_item_1024(*ctx, i);
        }
    };
    { std::vector<std::thread> ts; for (unsigned t = 0; t < threads; ++t) ts.emplace_back(fill); for (auto& t : ts) t.join(); }
    const double build_s = std::chrono::duration<double>(clk::now() - t0).count();

    ethash::hash256 header{};
    for (int i = 0; i < 32; ++i) header.bytes[i] = (uint8_t)(i * 7 + 1);
    ethash::hash256 impossible{};  // all-zero boundary: search never stops early

    // light-mode single-header verification cost (what CheckBlockHeader pays per header)
    const int nlight = 20;
    auto tl = clk::now();
    for (int i = 0; i < nlight; ++i) (void)progpow::hash(*static_cast<ethash_epoch_context*>(ctx), block, header, (uint64_t)i);
    const double light_ms = std::chrono::duration<double, std::milli>(clk::now() - tl).count() / nlight;

    // full-dataset search on every core, disjoint nonce ranges (the reference miner's layout)
    std::atomic<uint64_t> hashes{0};
    std::atomic<bool> stop{false};
    const size_t chunk = 2000;
    auto t1 = clk::now();
    auto worker = [&](unsigned t) {
        uint64_t nonce = (uint64_t)t << 40;
        while (!stop.load(std::memory_order_relaxed)) {
            (void)progpow::search(*ctx, block, header, impossible, nonce, chunk);
            nonce += chunk;
            hashes.fetch_add(chunk, std::memory_order_relaxed);
        }
    };
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < threads; ++t) ts.emplace_back(worker, t);
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    stop = true;
    for (auto& t : ts) t.join();
    const double el = std::chrono::duration<double>(clk::now() - t1).count();
    std::printf("{\"impl\": \"reference progpow::search (full dataset)\", \"epoch\": %d, \"dag_bytes\": %llu, "
                "\"threads\": %u, \"hashes\": %llu, \"seconds\": %.3f, \"mhs\": %.6f, \"light_hash_ms\": %.3f, "
                "\"dataset_fill_s\": %.1f}\n",
                epoch, (unsigned long long)n1024 * 128ull, threads, (unsigned long long)hashes.load(), el,
                hashes.load() / el / 1e6, light_ms, build_s);
    ethash_destroy_epoch_context_full(ctx);
    return 0;
}
