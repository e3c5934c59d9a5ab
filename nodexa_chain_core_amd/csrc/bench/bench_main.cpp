// bench_nodexa — host micro-benchmarks in the reference's bench_clore format.
//
// Parity: src/bench/bench.{h,cpp} (BENCHMARK registry, State::KeepRunning adaptive
// loop, CSV "#Benchmark,count,min,max,average"), src/bench/crypto_hash.cpp (1 MB
// buffers for RIPEMD160/SHA1/SHA256/SHA512, SHA256_32b, SipHash_32b) and the sample
// output the reference publishes in doc/benchmarking.md:12-22 — the only
// performance numbers in the reference. PoW benches are new: the
// reference has none (src/Makefile.bench.include:14-30).
//
//   bench_nodexa [-filter=<substring>] [-time=<seconds per bench>] [-list]
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../chain/script.hpp"
#include "../crypto/blake2b.hpp"
#include "../crypto/hashes.hpp"
#include "../crypto/keccak.hpp"
#include "../crypto/sha256.hpp"
#include "../pow/equihash.hpp"
#include "../pow/ethash.hpp"
#include "../pow/kawpow.hpp"
#include "../pow/x16r.hpp"
#include "../pow/x16r_prims.hpp"

namespace {

using Clock = std::chrono::steady_clock;

// Adaptive timing loop: batches grow until one batch takes >= budget/64, per-iteration
// min/max are taken over batches, the average over the whole run (as State::KeepRunning).
class State {
public:
    State(std::string name, double budget) : name_(std::move(name)), budget_(budget) {}
    bool keep_running() {
        if (!started_) {
            started_ = true;
            begin_ = last_ = Clock::now();
            in_batch_ = 1;
            return true;
        }
        if (in_batch_ < batch_) {
            ++in_batch_;
            return true;
        }
        const auto now = Clock::now();
        const double el = std::chrono::duration<double>(now - last_).count();
        if (el * 64 < budget_) {  // batch too short to time: grow it 8x and restart timing
            batch_ *= 8;
            count_ = 0;
            min_ = std::numeric_limits<double>::max();
            max_ = 0;
            begin_ = last_ = Clock::now();
            in_batch_ = 1;
            return true;
        }
        const double one = el / double(batch_);
        min_ = std::min(min_, one);
        max_ = std::max(max_, one);
        count_ += batch_;
        last_ = now;
        const double total = std::chrono::duration<double>(now - begin_).count();
        if (total < budget_) {
            in_batch_ = 1;
            return true;
        }
        std::printf("%s,%llu,%.15f,%.15f,%.15f\n", name_.c_str(), (unsigned long long)count_, min_, max_,
                    total / double(count_));
        std::fflush(stdout);
        return false;
    }

private:
    std::string name_;
    double budget_;
    Clock::time_point begin_, last_;
    bool started_ = false;
    unsigned long long batch_ = 1, in_batch_ = 0, count_ = 0;
    double min_ = std::numeric_limits<double>::max(), max_ = 0;
};

using Bench = std::function<void(State&)>;
std::map<std::string, Bench>& registry() {
    static std::map<std::string, Bench> r;
    return r;
}
struct Reg {
    Reg(const char* n, Bench b) { registry()[n] = std::move(b); }
};
#define BENCH(name) \
    static void bench_##name(State& state); \
    static Reg reg_##name(#name, bench_##name); \
    static void bench_##name(State& state)

using namespace nodexa;
constexpr size_t kBuf = 1000 * 1000;  // crypto_hash.cpp BUFFER_SIZE

BENCH(RIPEMD160) {
    std::vector<u8> in(kBuf, 0);
    u8 h[20];
    while (state.keep_running()) ripemd160(in.data(), in.size(), h);
}
BENCH(SHA1) {
    std::vector<u8> in(kBuf, 0);
    u8 h[20];
    while (state.keep_running()) sha1(in.data(), in.size(), h);
}
BENCH(SHA256) {
    std::vector<u8> in(kBuf, 0);
    u8 h[32];
    while (state.keep_running()) sha256(in.data(), in.size(), h);
}
BENCH(SHA256_32b) {
    u8 in[32] = {0};
    while (state.keep_running())
        for (int i = 0; i < 1000000; ++i) sha256(in, 32, in);
}
BENCH(SHA512) {
    std::vector<u8> in(kBuf, 0);
    while (state.keep_running()) {
        volatile u8 sink = sha512_hash(in.data(), in.size()).bytes[0];
        (void)sink;
    }
}
BENCH(SipHash_32b) {
    u8 v[32] = {0};
    u64 acc = 0;
    while (state.keep_running())
        for (int i = 0; i < 1000000; ++i) {
            acc += siphash_uint256(0x0706050403020100ULL, 0x0F0E0D0C0B0A0908ULL, v);
            v[0] = u8(acc);
        }
}
BENCH(Trig) {
    float sum = 0;
    u32 i = 0;
    while (state.keep_running()) sum += std::sin(float(++i) * 1e-3f);
    volatile float sink = sum;
    (void)sink;
}
BENCH(Keccak512_64b) {
    Hash512 h;
    while (state.keep_running()) h = keccak512(h.bytes, 64);
}
BENCH(BLAKE2b_Equihash_Row) {
    EquihashParams p;
    u8 input[140] = {0};
    Blake2b base = equihash_base_state(p, input, sizeof input);
    u8 out[25];
    u32 i = 0;
    while (state.keep_running()) equihash_leaf(p, base, i++ & 0xFFFFF, out);
}
BENCH(X16R_Header80) {
    u8 hdr[80] = {0}, out[32];
    for (int i = 0; i < 80; ++i) hdr[i] = u8(i * 7 + 1);
    while (state.keep_running()) {
        x16r_hash(hdr, 80, hdr + 4, false, out);
        ++hdr[76];
    }
}
BENCH(X16RV2_Header80) {
    u8 hdr[80] = {0}, out[32];
    for (int i = 0; i < 80; ++i) hdr[i] = u8(i * 11 + 3);
    while (state.keep_running()) {
        x16r_hash(hdr, 80, hdr + 4, true, out);
        ++hdr[76];
    }
}
BENCH(KAWPOW_HashNoVerify) {
    Hash256 hh, mix;
    u64 nonce = 0;
    while (state.keep_running()) hh = kawpow_hash_no_verify(30000, hh, mix, nonce++);
}
BENCH(KAWPOW_HashLight_epoch0) {
    // CheckBlockHeader -> GetHashFull: the per-header cost of the reference's serial verify
    auto ctx = get_epoch_context(0);
    Hash256 hh;
    u64 nonce = 0;
    while (state.keep_running()) {
        KawpowResult r = kawpow_hash(*ctx, 1000, hh, nonce++);
        hh.bytes[0] ^= r.final_hash.bytes[0];
    }
}
BENCH(Equihash_200_9_Verify) {
    EquihashParams p;
    u8 input[140] = {0};
    std::vector<std::vector<u32>> sols;
    for (u32 k = 0; sols.empty() && k < 64; ++k) {
        store_le32(input + 108, k);
        sols = equihash_solve_cpu(p, input, sizeof input, 1, nullptr, 0);
    }
    if (sols.empty()) return;
    while (state.keep_running())
        if (!equihash_verify(p, input, sizeof input, sols[0])) std::abort();
}

}  // namespace

int main(int argc, char** argv) {
    std::string filter;
    double budget = 1.0;
    bool list = false;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a.rfind("-filter=", 0) == 0) filter = a.substr(8);
        else if (a.rfind("-time=", 0) == 0) budget = std::stod(a.substr(6));
        else if (a == "-list") list = true;
        else {
            std::fprintf(stderr, "usage: bench_nodexa [-filter=<substr>] [-time=<s>] [-list]\n");
            return 2;
        }
    }
    if (list) {
        for (auto& kv : registry()) std::printf("%s\n", kv.first.c_str());
        return 0;
    }
    std::printf("#Benchmark,count,min,max,average\n");
    for (auto& kv : registry())
        if (filter.empty() || kv.first.find(filter) != std::string::npos) {
            State st(kv.first, budget);
            kv.second(st);
        }
    return 0;
}
