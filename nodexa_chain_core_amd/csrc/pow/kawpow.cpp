#include "kawpow.hpp"

#include <algorithm>
#include <chrono>
#include <thread>

namespace nodexa {

namespace {

// "rAVENCOINKAWPOW", one byte per u32 word (progpow.cpp:157-173; note the
// lowercase 'r').
constexpr u32 kKawpowPad[15] = {0x72, 0x41, 0x56, 0x45, 0x4E, 0x43, 0x4F, 0x49,
                                0x4E, 0x4B, 0x41, 0x57, 0x50, 0x4F, 0x57};

inline void run_lane_program(const KawpowProgram& p, u32* m, const u32* l1) {
    for (int i = 0; i < kNumMathOps; ++i) {
        if (i < kNumCacheAccesses) {
            const auto& c = p.cache[i];
            kawpow_merge(m[c.dst], l1[m[c.src] % kL1CacheWords], c.sel);
        }
        const auto& o = p.math[i];
        kawpow_merge(m[o.dst], kawpow_math(m[o.src1], m[o.src2], o.sel1), o.sel2);
    }
}

template <typename Lookup>
Hash256 hash_mix(const KawpowProgram& prog, u32 full_items, const u32* l1, const u32 seed[2],
                 Lookup&& lookup) {
    u32 mix[kNumLanes][kNumRegs];
    const u32 z = fnv1a(kFnvOffsetBasis, seed[0]);
    const u32 w = fnv1a(z, seed[1]);
    for (u32 l = 0; l < kNumLanes; ++l) {
        const u32 jsr = fnv1a(w, l);
        Kiss99 rng{z, w, jsr, fnv1a(jsr, l)};
        for (int i = 0; i < kNumRegs; ++i) mix[l][i] = rng();
    }
    const u32 num_items = full_items / 2;
    Hash512 item[4];
    for (u32 r = 0; r < kNumRounds; ++r) {
        const u32 index = mix[r % kNumLanes][0] % num_items;
        lookup(index, item);
        const u32* words = item[0].w32;  // 64 contiguous words (item is a Hash512[4])
        for (u32 l = 0; l < kNumLanes; ++l) {
            run_lane_program(prog, mix[l], l1);
            const u32 off = ((l ^ r) % kNumLanes) * kDagLoads;
            for (int i = 0; i < kDagLoads; ++i) kawpow_merge(mix[l][prog.dag_dst[i]], words[off + i], prog.dag_sel[i]);
        }
    }
    Hash256 out;
    for (int i = 0; i < 8; ++i) out.w32[i] = kFnvOffsetBasis;
    for (u32 l = 0; l < kNumLanes; ++l) {
        u32 h = kFnvOffsetBasis;
        for (int i = 0; i < kNumRegs; ++i) h = fnv1a(h, mix[l][i]);
        out.w32[l % 8] = fnv1a(out.w32[l % 8], h);
    }
    return out;
}

}  // namespace

KawpowProgram make_kawpow_program(u64 period) {
    KawpowProgram p;
    p.period = period;
    const u32 lo = u32(period), hi = u32(period >> 32);
    const u32 z = fnv1a(kFnvOffsetBasis, lo);
    const u32 w = fnv1a(z, hi);
    const u32 jsr = fnv1a(w, lo);
    Kiss99 rng{z, w, jsr, fnv1a(jsr, hi)};
    u32 dst_seq[kNumRegs], src_seq[kNumRegs];
    for (u32 i = 0; i < kNumRegs; ++i) dst_seq[i] = src_seq[i] = i;
    for (u32 i = kNumRegs; i > 1; --i) {
        std::swap(dst_seq[i - 1], dst_seq[rng() % i]);
        std::swap(src_seq[i - 1], src_seq[rng() % i]);
    }
    u32 dst_ctr = 0, src_ctr = 0;
    auto next_dst = [&] { return dst_seq[(dst_ctr++) % kNumRegs]; };
    auto next_src = [&] { return src_seq[(src_ctr++) % kNumRegs]; };
    for (int i = 0; i < kNumMathOps; ++i) {
        if (i < kNumCacheAccesses) {
            auto& c = p.cache[i];
            c.src = u8(next_src());
            c.dst = u8(next_dst());
            c.sel = rng();
        }
        auto& o = p.math[i];
        const u32 src_rnd = rng() % (kNumRegs * (kNumRegs - 1));
        o.src1 = u8(src_rnd % kNumRegs);
        u32 src2 = src_rnd / kNumRegs;
        if (src2 >= o.src1) ++src2;
        o.src2 = u8(src2);
        o.sel1 = rng();
        o.dst = u8(next_dst());
        o.sel2 = rng();
    }
    for (int i = 0; i < kDagLoads; ++i) {
        p.dag_dst[i] = u8(i == 0 ? 0 : next_dst());
        p.dag_sel[i] = rng();
    }
    return p;
}

void kawpow_initial_state(const Hash256& header_hash, u64 nonce, u32 state2[8]) {
    u32 st[25];
    for (int i = 0; i < 8; ++i) st[i] = header_hash.w32[i];
    st[8] = u32(nonce);
    st[9] = u32(nonce >> 32);
    for (int i = 10; i < 25; ++i) st[i] = kKawpowPad[i - 10];
    keccakf800(st);
    for (int i = 0; i < 8; ++i) state2[i] = st[i];
}

Hash256 kawpow_final(const u32 state2[8], const Hash256& mix_hash) {
    u32 st[25];
    for (int i = 0; i < 8; ++i) st[i] = state2[i];
    for (int i = 0; i < 8; ++i) st[8 + i] = mix_hash.w32[i];
    for (int i = 16; i < 25; ++i) st[i] = kKawpowPad[i - 16];
    keccakf800(st);
    Hash256 out;
    for (int i = 0; i < 8; ++i) out.w32[i] = st[i];
    return out;
}

namespace {
// One program per period; a tiny cache keeps the most recent period hot.
const KawpowProgram& program_for(int block_number, KawpowProgram& slot) {
    const u64 period = kawpow_period(block_number);
    if (slot.period != period) slot = make_kawpow_program(period);
    return slot;
}
}  // namespace

KawpowResult kawpow_hash(const EpochContext& ctx, int block_number, const Hash256& header_hash,
                         u64 nonce) {
    thread_local KawpowProgram prog_slot{};
    const KawpowProgram& prog = program_for(block_number, prog_slot);
    u32 state2[8];
    kawpow_initial_state(header_hash, nonce, state2);
    KawpowResult r;
    r.mix_hash = hash_mix(prog, u32(ctx.full_items), ctx.l1.data(), state2,
                          [&](u32 index, Hash512* item) { dataset_item_2048(ctx, index, item); });
    r.final_hash = kawpow_final(state2, r.mix_hash);
    return r;
}

KawpowResult kawpow_hash_full(HostDag& dag, int block_number, const Hash256& header_hash, u64 nonce) {
    thread_local KawpowProgram prog_slot{};
    const KawpowProgram& prog = program_for(block_number, prog_slot);
    u32 state2[8];
    kawpow_initial_state(header_hash, nonce, state2);
    KawpowResult r;
    r.mix_hash = hash_mix(prog, u32(dag.ctx().full_items), dag.ctx().l1.data(), state2,
                          [&](u32 index, Hash512* item) { dag.item2048(index, item); });
    r.final_hash = kawpow_final(state2, r.mix_hash);
    return r;
}

bool kawpow_verify(const EpochContext& ctx, int block_number, const Hash256& header_hash,
                   const Hash256& mix_hash, u64 nonce, const Hash256& boundary) {
    u32 state2[8];
    kawpow_initial_state(header_hash, nonce, state2);
    if (!hash_le(kawpow_final(state2, mix_hash), boundary)) return false;
    thread_local KawpowProgram prog_slot{};
    const KawpowProgram& prog = program_for(block_number, prog_slot);
    const Hash256 expected = hash_mix(prog, u32(ctx.full_items), ctx.l1.data(), state2,
                                      [&](u32 index, Hash512* item) { dataset_item_2048(ctx, index, item); });
    return expected == mix_hash;
}

Hash256 kawpow_hash_no_verify(int /*block_number*/, const Hash256& header_hash, const Hash256& mix_hash,
                              u64 nonce) {
    u32 state2[8];
    kawpow_initial_state(header_hash, nonce, state2);
    return kawpow_final(state2, mix_hash);
}

KawpowSearchResult kawpow_search_light(const EpochContext& ctx, int block_number,
                                       const Hash256& header_hash, const Hash256& boundary,
                                       u64 start_nonce, u64 iterations) {
    KawpowSearchResult out;
    for (u64 n = start_nonce; n < start_nonce + iterations; ++n) {
        KawpowResult r = kawpow_hash(ctx, block_number, header_hash, n);
        if (hash_le(r.final_hash, boundary)) {
            out.found = true;
            out.nonce = n;
            out.result = r;
            return out;
        }
    }
    return out;
}

KawpowSearchResult kawpow_search_full(HostDag& dag, int block_number, const Hash256& header_hash,
                                      const Hash256& boundary, u64 start_nonce, u64 iterations,
                                      int threads) {
    if (threads <= 0) threads = int(std::max(1u, std::thread::hardware_concurrency()));
    std::atomic<u64> next{0};
    std::atomic<u64> best{~0ULL};
    std::mutex mu;
    KawpowSearchResult out;
    const u64 chunk = 64;
    auto worker = [&] {
        for (;;) {
            const u64 lo = next.fetch_add(chunk);
            if (lo >= iterations || lo > best.load()) break;
            const u64 hi = std::min(iterations, lo + chunk);
            for (u64 i = lo; i < hi; ++i) {
                const u64 n = start_nonce + i;
                KawpowResult r = kawpow_hash_full(dag, block_number, header_hash, n);
                if (hash_le(r.final_hash, boundary)) {
                    std::lock_guard<std::mutex> g(mu);
                    if (i < best.load()) {
                        best.store(i);
                        out.found = true;
                        out.nonce = n;
                        out.result = r;
                    }
                    break;
                }
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) pool.emplace_back(worker);
    for (auto& t : pool) t.join();
    return out;
}

double kawpow_cpu_hashrate(HostDag& dag, int block_number, u64 nonces, int threads) {
    if (threads <= 0) threads = int(std::max(1u, std::thread::hardware_concurrency()));
    Hash256 header;
    header.w32[0] = 0x12345678;
    std::atomic<u64> next{0};
    std::atomic<u32> sink{0};
    auto worker = [&] {
        u32 acc = 0;
        for (;;) {
            const u64 i = next.fetch_add(1);
            if (i >= nonces) break;
            acc ^= kawpow_hash_full(dag, block_number, header, i).final_hash.w32[0];
        }
        sink ^= acc;
    };
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) pool.emplace_back(worker);
    for (auto& t : pool) t.join();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return double(nonces) / dt;
}

}  // namespace nodexa
