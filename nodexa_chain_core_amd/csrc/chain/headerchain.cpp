#include "headerchain.hpp"

#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <thread>
#include <unordered_set>

#include "../pow/equihash.hpp"
#include "../pow/kawpow.hpp"
#include "../pow/x16r.hpp"
#include "../util/workpool.hpp"

namespace nodexa {

// ---------------------------------------------------------------- verifier
Uint256 CpuPowVerifier::block_hash(const BlockHeader& h, const ChainParams& p) const {
    if (h.is_equihash()) return h.equihash_hash(p.kawpow_activation_time);  // SHA256d(header) (extension)
    switch (p.algo_for(h.time)) {
        case PowAlgo::KAWPOW: {
            const Hash256 fin = kawpow_hash_no_verify(int(h.height), h.kawpow_header_hash().to_progpow(),
                                                      h.mix_hash.to_progpow(), h.nonce64);
            return Uint256::from_progpow(fin);
        }
        case PowAlgo::X16RV2:
        case PowAlgo::X16R: {
            const Bytes d = h.legacy80();
            Uint256 out;
            x16r_hash(d.data(), d.size(), h.prev.data, p.algo_for(h.time) == PowAlgo::X16RV2, out.data);
            return out;
        }
    }
    return Uint256();
}

Uint256 CpuPowVerifier::block_hash_full(const BlockHeader& h, const ChainParams& p, Uint256& mix) const {
    if (h.is_equihash() || p.algo_for(h.time) != PowAlgo::KAWPOW) {
        mix = Uint256();
        return block_hash(h, p);
    }
    auto ctx = get_epoch_context(epoch_of_block(int(h.height)));
    const KawpowResult r = kawpow_hash(*ctx, int(h.height), h.kawpow_header_hash().to_progpow(), h.nonce64);
    mix = Uint256::from_progpow(r.mix_hash);
    return Uint256::from_progpow(r.final_hash);
}

// ---------------------------------------------------------------- chain
namespace {

// GetSkipHeight (src/chain.cpp): the height an entry's skip pointer targets
int skip_height(int h) {
    auto invert_low = [](int n) { return n & (n - 1); };
    return h < 2 ? 0 : ((h & 1) ? invert_low(invert_low(h - 1)) + 1 : invert_low(h));
}

}  // namespace

HeaderChain::HeaderChain(ChainParams params, std::shared_ptr<const PowVerifier> verifier)
    : params_(std::move(params)), verifier_(std::move(verifier)) {
    const BlockHeader& g = params_.genesis.header;
    Uint256 gh = params_.consensus.genesis_hash;
    if (gh.is_null()) gh = verifier_->block_hash(g, params_);
    params_.consensus.genesis_hash = gh;
    genesis_ = add_to_index(g, gh, nullptr);
    update_active_chain();
}

const HeaderIndex* HeaderChain::add_to_index(const BlockHeader& h, const Uint256& hash, const HeaderIndex* prev,
                                              const ArithU256* proof, const std::vector<const HeaderIndex*>* batch) {
    HeaderIndex& idx = *storage_.alloc();
    idx.hash = hash;
    idx.prev = prev;
    idx.height = prev ? prev->height + 1 : 0;
    idx.time = h.time;
    idx.bits = h.bits;
    idx.header = h;
    idx.chain_work = (prev ? prev->chain_work : ArithU256()) + (proof ? *proof : block_proof(h.bits));
    if (prev) {
        const int skip_h = skip_height(idx.height);
        // inside a linear batch the skip target is often a node added moments ago: look it up
        // directly instead of walking back from prev
        const int b0 = batch && !batch->empty() ? (*batch)[0]->height : 0;
        idx.skip = batch && !batch->empty() && skip_h >= b0 ? (*batch)[size_t(skip_h - b0)] : prev->ancestor(skip_h);
    }
    index_.insert(&idx);
    ++version_;
    return &idx;
}

AcceptResult HeaderChain::check_header(const BlockHeader& h, bool check_pow) const {
    AcceptResult r;
    if (!check_pow) {
        r.ok = true;
        return r;
    }
    if (h.is_equihash()) {
        // extension: valid (n,k) solution for kawpow_input || nonce256, then
        // SHA256d(header) <= target
        const EquihashParams ep{params_.equihash_n, params_.equihash_k};
        const Bytes in = h.equihash_input();
        if (int(h.solution.size()) != ep.solution_bytes() ||
            !equihash_verify(ep, in.data(), in.size(), equihash_unpack_indices(ep, h.solution))) {
            r.reject = "invalid-solution";
            r.dos = 100;
            return r;
        }
        if (!check_proof_of_work(verifier_->block_hash(h, params_), h.bits, params_)) {
            r.reject = "high-hash";
            r.dos = 50;
            return r;
        }
        r.ok = true;
        return r;
    }
    const bool kawpow = h.time >= params_.kawpow_activation_time;
    if (kawpow) {
        const int cp = params_.last_checkpoint_height();
        if (cp >= 0 && int64_t(h.height) <= cp) {
            if (!check_proof_of_work(verifier_->block_hash(h, params_), h.bits, params_)) {
                r.reject = "high-hash";
                r.dos = 50;
                return r;
            }
            r.ok = true;
            return r;
        }
    }
    Uint256 mix;
    const Uint256 pow = verifier_->block_hash_full(h, params_, mix);
    if (!check_proof_of_work(pow, h.bits, params_)) {
        r.reject = "high-hash";
        r.dos = 50;
        return r;
    }
    if (kawpow && mix != h.mix_hash) {
        r.reject = "invalid-mix-hash";
        r.dos = 50;
        return r;
    }
    r.ok = true;
    return r;
}

u32 HeaderChain::next_bits(const BlockHeader& candidate) const {
    std::lock_guard<std::recursive_mutex> g(mu_);
    return next_work_required(tip(), candidate, params_);
}

AcceptResult HeaderChain::accept_header(const BlockHeader& h, int64_t adjusted_time, bool check_pow) {
    return accept_header_impl(h, nullptr, adjusted_time, check_pow, nullptr, nullptr);
}

// ContextualCheckBlockHeader after the -maxreorg guard, in the reference's order, on values the
// caller supplies: the expected nBits, the parent's median time past and whether the header forks
// below the last checkpoint (the only rule that reads the active chain). Context-free otherwise,
// so a linear batch evaluates it for all headers at once.
bool HeaderChain::contextual_rules(const BlockHeader& h, const Uint256& hash, int height, u32 expected_bits,
                                   int64_t prev_mtp, int64_t adjusted_time, bool cp_fork, AcceptResult& r) const {
    if (h.bits != expected_bits) {
        r.reject = "bad-diffbits";
        r.dos = 100;
        return false;
    }
    if (cp_fork) {
        r.reject = "bad-fork-prior-to-checkpoint";
        r.dos = 100;
        return false;
    }
    auto cpit = params_.checkpoints.find(height);
    if (cpit != params_.checkpoints.end() && cpit->second != hash) {
        r.reject = "checkpoint mismatch";
        r.dos = 100;
        return false;
    }
    if (int64_t(h.time) <= prev_mtp) {
        r.reject = "time-too-old";
        return false;
    }
    const int64_t max_future = (height >= params_.dgw_activation_block) ? kMaxFutureBlockTimeDgw : kMaxFutureBlockTime;
    if (int64_t(h.time) > adjusted_time + max_future) {
        r.reject = "time-too-new";
        return false;
    }
    if (h.version < kVersionBitsTopBitsAssets) {
        char buf[48];
        std::snprintf(buf, sizeof(buf), "bad-version(0x%08x)", unsigned(h.version));
        r.reject = buf;
        return false;
    }
    // Equihash extension era (new): the flag bit is required from the activation
    // time on and forbidden before it (so reference-network headers never parse
    // as extended ones), and the extended header commits to its height.
    const bool eq_era = h.time >= params_.equihash_activation_time;
    if (eq_era != h.is_equihash()) {
        r.reject = eq_era ? "bad-version(equihash-required)" : "bad-version(equihash-not-active)";
        r.dos = 100;
        return false;
    }
    if (h.is_equihash() && int(h.height) != height) {
        r.reject = "bad-height";
        r.dos = 100;
        return false;
    }
    // The reference never checks that a KawPow header's nHeight equals its index
    // height (the epoch/period therefore follow the claimed height). Off by
    // default for consensus compatibility; -strictheight turns it on as policy.
    if (strict_kawpow_height && params_.algo_for(h.time) == PowAlgo::KAWPOW && int(h.height) != height) {
        r.reject = "bad-height";
        r.dos = 100;
        return false;
    }
    return true;
}

AcceptResult HeaderChain::accept_header_impl(const BlockHeader& h, const Uint256* known_hash, int64_t adjusted_time,
                                             bool check_pow, const u32* expected_bits, const AcceptResult* precheck,
                                             const ArithU256* proof, const int64_t* prev_mtp) {
    std::lock_guard<std::recursive_mutex> g(mu_);
    AcceptResult r;
    const Uint256 hash = known_hash ? *known_hash : verifier_->block_hash(h, params_);
    if (hash == params_.consensus.genesis_hash) {
        r.ok = true;
        r.duplicate = true;
        r.index = genesis_;
        return r;
    }
    if (const HeaderIndex* self = index_.find(hash)) {
        r.index = self;
        r.duplicate = true;
        if (failed_.count(self)) {
            r.reject = "duplicate";
            return r;
        }
        r.ok = true;
        return r;
    }
    r = precheck ? *precheck : check_header(h, check_pow);
    if (!r.ok) return r;
    r.ok = false;
    const HeaderIndex* prev = index_.find(h.prev);
    if (prev == nullptr) {
        r.reject = "prev-blk-not-found";
        r.dos = 10;
        return r;
    }
    if (failed_.count(prev)) {
        r.reject = "bad-prevblk";
        r.dos = 100;
        return r;
    }
    // ContextualCheckBlockHeader
    const int height = prev->height + 1;
    if (max_reorg_depth > 0 && this->height() - (height - 1) >= max_reorg_depth) {
        r.reject = "bad-fork-prior-to-maxreorgdepth";
        r.dos = 10;
        return r;
    }
    const int cp = params_.last_checkpoint_height();
    const bool cp_fork = cp >= 0 && height < cp && at_height(cp) != nullptr;
    if (!contextual_rules(h, hash, height, expected_bits ? *expected_bits : next_work_required(prev, h, params_),
                          prev_mtp ? *prev_mtp : prev->median_time_past(), adjusted_time, cp_fork, r))
        return r;
    r.index = add_to_index(h, hash, prev, proof);
    r.ok = true;
    consider_new_header(r.index);
    return r;
}

namespace {

template <class F>
void parallel_for(size_t n, F&& fn) {
    parallel_for_each(n, fn, 128);  // the persistent pool (util/workpool.hpp): no thread spawn per call
}

}  // namespace

// ProcessNewBlockHeaders. For a batch that extends a known header linearly (the shape of
// every P2P `headers` message) the block hashes and the expected nBits of all headers
// are computed up front on all host cores: DarkGravityWave only reads the 180 previous
// (nTime, nBits) pairs, which the batch itself supplies, so header i's retarget does not
// wait for header i-1 to be indexed. The serial pass then does the index updates and
// the remaining contextual checks. Results are identical to accepting one by one.
bool HeaderChain::dgw_series(const BlockHeader* hs, size_t n, const Uint256* hashes, std::vector<u32>& times,
                             std::vector<u32>& bits, size_t& a, int& base_height) const {
    std::lock_guard<std::recursive_mutex> g(mu_);
    if (n == 0 || hashes == nullptr) return false;
    const HeaderIndex* base = index_.find(hs[0].prev);
    bool linear = base != nullptr;
    for (size_t i = 1; linear && i < n; ++i) linear = hs[i].prev == hashes[i - 1];
    const ConsensusParams& c = params_.consensus;
    if (!linear || (c.pow_allow_min_difficulty_blocks && c.pow_no_retargeting)) return false;
    std::vector<const HeaderIndex*> anc;  // base and up to 179 ancestors, newest first
    for (const HeaderIndex* p = base; p && anc.size() < size_t(kDgwPastBlocks); p = p->prev) anc.push_back(p);
    a = anc.size();
    base_height = base->height;
    times.assign(a + n, 0);
    bits.assign(a + n, 0);
    for (size_t k = 0; k < a; ++k) {
        times[k] = anc[a - 1 - k]->time;
        bits[k] = anc[a - 1 - k]->bits;
    }
    for (size_t i = 0; i < n; ++i) {
        times[a + i] = hs[i].time;
        bits[a + i] = hs[i].bits;
    }
    return true;
}

std::vector<AcceptResult> HeaderChain::accept_headers(const std::vector<BlockHeader>& hs, int64_t adjusted_time,
                                                      bool check_pow, const std::vector<Uint256>* known_hashes,
                                                      const std::vector<u32>* known_bits) {
    return accept_headers(hs.data(), hs.size(), adjusted_time, check_pow,
                          known_hashes && known_hashes->size() == hs.size() ? known_hashes->data() : nullptr,
                          known_bits && known_bits->size() == hs.size() ? known_bits->data() : nullptr);
}

// out[k] = base + proofs[0] + ... + proofs[k] (mod 2^256): the chain work of a run of headers,
// in 64-bit limbs with the carries chained (one 256-bit add is four adds, not eight).
static void chain_work_prefix(const ArithU256& base, const ArithU256* proofs, size_t m, ArithU256* out) {
    u64 acc[4], p[4];
    std::memcpy(acc, base.pn, 32);
    for (size_t k = 0; k < m; ++k) {
        std::memcpy(p, proofs[k].pn, 32);
        unsigned __int128 s = (unsigned __int128)acc[0] + p[0];
        acc[0] = u64(s);
        s = (unsigned __int128)acc[1] + p[1] + u64(s >> 64);
        acc[1] = u64(s);
        s = (unsigned __int128)acc[2] + p[2] + u64(s >> 64);
        acc[2] = u64(s);
        acc[3] = acc[3] + p[3] + u64(s >> 64);
        std::memcpy(out[k].pn, acc, 32);
    }
}

std::vector<AcceptResult> HeaderChain::accept_headers(const BlockHeader* hs, size_t n, int64_t adjusted_time,
                                                      bool check_pow, const Uint256* known_hashes,
                                                      const u32* known_bits) {
    std::lock_guard<std::recursive_mutex> g(mu_);
    AcceptPrep p = prepare_headers(hs, n, adjusted_time, check_pow, known_hashes, known_bits);
    return commit_headers(p, n);
}

AcceptPrep HeaderChain::prepare_headers(const BlockHeader* hs, size_t n, int64_t adjusted_time, bool check_pow,
                                        const Uint256* known_hashes, const u32* known_bits) const {
    std::lock_guard<std::recursive_mutex> g(mu_);
    AcceptPrep P;
    P.hs = hs;
    P.n = n;
    P.adjusted_time = adjusted_time;
    P.check_pow = check_pow;
    P.version = version_;
    P.strict_height = strict_kawpow_height;
    if (known_bits) P.known_bits.assign(known_bits, known_bits + n);
    std::vector<Uint256>& hashes = P.hashes;
    std::vector<u32>& expected = P.expected;
    std::vector<u8>& have = P.have;
    std::vector<u8>& have_mtp = P.have_mtp;
    have.assign(n, 0);
    have_mtp.assign(n, 0);
    std::vector<ArithU256>& proofs = P.proofs;
    std::vector<int64_t>& mtp = P.mtp;
    std::vector<AcceptResult>& pre = P.pre;
    if (n >= kParallelAcceptMin && check_pow) {  // CheckBlockHeader (full PoW) is context-free
        pre.resize(n);
        parallel_for(n, [&](size_t i) { pre[i] = check_header(hs[i], true); });
    }
    std::vector<u8>& ctx = P.ctx;
    std::vector<u8>& fresh = P.fresh;
    int& base_height = P.base_height;
    if (n >= kParallelAcceptMin) {
        if (known_hashes) {
            hashes.assign(known_hashes, known_hashes + n);
        } else {
            hashes.resize(n);
            parallel_for(n, [&](size_t i) { hashes[i] = verifier_->block_hash(hs[i], params_); });
        }
        // The context-free per-header work of the serial pass, done up front in one pass on all
        // cores: the block proof (2^256 / (target + 1)) and, for a linear batch, the parent's
        // median time past and the expected nBits from the batch's own (nTime, nBits) series --
        // and then, when nothing in the index has failed, the contextual rules themselves
        // (ctx: 1 ok, 0 failed or not evaluated, 2 failed at bad-diffbits) and whether the header
        // is new to the index (a linear batch cannot repeat a hash).
        proofs.resize(n);
        std::vector<u32> times, bits;
        size_t a = 0;
        if (!dgw_series(hs, n, hashes.data(), times, bits, a, base_height)) {
            parallel_for(n, [&](size_t i) { proofs[i] = block_proof(hs[i].bits); });
        } else {
            const bool from_genesis = a == size_t(base_height) + 1;  // the series reaches genesis
            const bool fast = failed_.empty() && !(check_pow && pre.empty());
            const u32 limit_compact = ArithU256::from_uint256(params_.consensus.pow_limit).get_compact();
            mtp.assign(n, 0);
            expected.assign(n, 0);
            if (fast) {
                ctx.assign(n, 0);
                fresh.assign(n, 0);
            }
            parallel_for(n, [&](size_t i) {
                proofs[i] = block_proof(hs[i].bits);
                const int64_t j = int64_t(a) - 1 + int64_t(i);  // series index of header i's parent
                if (j >= 10 || from_genesis) {
                    int64_t w[11];
                    int m = 0;
                    for (int64_t k = j; k >= 0 && m < 11; --k) w[m++] = times[size_t(k)];
                    std::sort(w, w + m);
                    mtp[i] = w[m / 2];
                    have_mtp[i] = 1;
                }
                // expected nBits: from the caller where it has them (the GPU batch kernel, dgw.hip,
                // computes them from the same series; 0 = not computed there), else from the
                // series here; BTC-retarget-era headers are left to the serial path
                const int last_height = base_height + int(i);  // height of header i's parent
                if (known_bits && known_bits[i] != 0) {
                    expected[i] = known_bits[i];
                    have[i] = 1;
                } else if (last_height + 1 >= params_.dgw_activation_block) {
                    expected[i] = last_height < kDgwPastBlocks
                                      ? limit_compact
                                      : dgw_average(times.data(), bits.data(), j, hs[i].time, params_);
                    have[i] = 1;
                }
                if (!fast) return;
                fresh[i] = index_.find(hashes[i]) == nullptr;
                if (!have[i] || !have_mtp[i]) return;
                AcceptResult r;
                ctx[i] = contextual_rules(hs[i], hashes[i], last_height + 1, expected[i], mtp[i], adjusted_time, false, r)
                             ? 1
                             : (r.reject == "bad-diffbits" ? 2 : 0);
            });
        }
    }
    return P;
}

std::vector<AcceptResult> HeaderChain::commit_headers(AcceptPrep& P, size_t hi) {
    std::lock_guard<std::recursive_mutex> g(mu_);
    hi = std::min(hi, P.n);
    if (P.version != version_ || P.strict_height != strict_kawpow_height) {
        // the index (or the height policy) changed since the prepare: prepare the prefix again
        AcceptPrep again = prepare_headers(P.hs, hi, P.adjusted_time, P.check_pow,
                                           P.hashes.size() >= hi ? P.hashes.data() : nullptr,
                                           P.known_bits.size() >= hi ? P.known_bits.data() : nullptr);
        return commit_headers(again, hi);
    }
    const BlockHeader* hs = P.hs;
    const size_t n = hi;
    const int64_t adjusted_time = P.adjusted_time;
    const bool check_pow = P.check_pow;
    std::vector<Uint256>& hashes = P.hashes;
    std::vector<u32>& expected = P.expected;
    std::vector<u8>& have = P.have;
    std::vector<u8>& have_mtp = P.have_mtp;
    std::vector<ArithU256>& proofs = P.proofs;
    std::vector<int64_t>& mtp = P.mtp;
    std::vector<AcceptResult>& pre = P.pre;
    std::vector<u8>& ctx = P.ctx;
    std::vector<u8>& fresh = P.fresh;
    const int base_height = P.base_height;
    std::vector<AcceptResult> out;
    out.reserve(n);
    if (ctx.empty()) {
        for (size_t i = 0; i < n; ++i) {
            out.push_back(accept_header_impl(hs[i], hashes.empty() ? nullptr : &hashes[i], adjusted_time, check_pow,
                                             have[i] ? &expected[i] : nullptr, pre.empty() ? nullptr : &pre[i],
                                             proofs.empty() ? nullptr : &proofs[i], have_mtp[i] ? &mtp[i] : nullptr));
            if (!out.back().ok) break;
        }
        return out;
    }
    // A linear batch with nothing failed in the index (every P2P `headers` message of a syncing
    // node): one serial pass does only what needs the index -- the duplicate and -maxreorg
    // checks, the checkpoint-fork rule, the insert (parent = the header just added, skip pointers
    // from the batch) and the tip extension. Same results and reject reasons as
    // accept_header_impl per header.
    index_.reserve(index_.size() + n);
    const int cp = params_.last_checkpoint_height();
    std::vector<const HeaderIndex*> batch;  // batch[k]: the index entry at height base_height + 1 + k
    batch.reserve(n);
    out.resize(n);
    std::vector<HeaderIndex*> nodes;
    std::vector<ArithU256> work;
    const HeaderIndex* prev = index_.find(hs[0].prev);
    size_t i = 0;
    while (i < n) {
        // A run of new headers that pass every rule on top of the active tip becomes the tip one
        // header after another (the -maxreorg and checkpoint-fork rules cannot fire on a header
        // whose parent is the tip): the entries are filled on all cores, only the chain-work
        // prefix sum, the table inserts and the active-chain append stay serial.
        size_t m = 0;
        if (!active_.empty() && prev == active_.back())
            while (i + m < n && fresh[i + m] && ctx[i + m] == 1 && (pre.empty() || pre[i + m].ok) &&
                   !(hashes[i + m] == params_.consensus.genesis_hash))
                ++m;
        if (m > 0) {
            const size_t s0 = batch.size();
            nodes.resize(m);
            work.resize(m);
            chain_work_prefix(prev->chain_work, proofs.data() + i, m, work.data());
            storage_.emplace_n(m, nodes.data(), [&] {
                batch.insert(batch.end(), nodes.begin(), nodes.end());  // reserved: no reallocation
                parallel_for(m, [&](size_t k) {
                    HeaderIndex& e = *new (nodes[k]) HeaderIndex();
                    const size_t j = i + k;
                    e.hash = hashes[j];
                    e.prev = k ? nodes[k - 1] : prev;
                    e.height = base_height + 1 + int(j);
                    e.time = hs[j].time;
                    e.bits = hs[j].bits;
                    e.header = hs[j];
                    e.chain_work = work[k];
                    const int sh = skip_height(e.height);
                    e.skip = sh > base_height ? batch[size_t(sh - base_height - 1)] : prev->ancestor(sh);
                    index_.insert_concurrent(&e);
                    out[j].ok = true;
                    out[j].index = &e;
                });
            });
            index_.add_count(m);
            ++version_;
            active_.insert(active_.end(), batch.begin() + std::ptrdiff_t(s0), batch.end());
            prev = batch.back();
            i += m;
            continue;
        }
        AcceptResult& r = out[i];
        if (!have[i] || !have_mtp[i] || hashes[i] == params_.consensus.genesis_hash) {
            r = accept_header_impl(hs[i], &hashes[i], adjusted_time, check_pow, have[i] ? &expected[i] : nullptr,
                                   pre.empty() ? nullptr : &pre[i], &proofs[i], have_mtp[i] ? &mtp[i] : nullptr);
            if (!r.ok) break;
            batch.push_back(prev = r.index);
            ++i;
            continue;
        }
        if (!fresh[i]) {  // already indexed (failed_ is empty: never "duplicate")
            r.ok = r.duplicate = true;
            r.index = prev = index_.find(hashes[i]);
            batch.push_back(prev);
            ++i;
            continue;
        }
        const int height = base_height + 1 + int(i);
        if (!pre.empty() && !pre[i].ok) {
            r = pre[i];
        } else if (max_reorg_depth > 0 && int(active_.size()) - 1 - (height - 1) >= max_reorg_depth) {
            r.reject = "bad-fork-prior-to-maxreorgdepth";
            r.dos = 10;
        } else if (ctx[i] != 1) {
            const bool cp_fork = ctx[i] == 0 && cp >= 0 && height < cp && size_t(cp) < active_.size();
            contextual_rules(hs[i], hashes[i], height, expected[i], mtp[i], adjusted_time, cp_fork, r);
        } else if (cp >= 0 && height < cp && size_t(cp) < active_.size()) {
            r.reject = "bad-fork-prior-to-checkpoint";
            r.dos = 100;
        } else {  // passes, but off the active tip (a fork): the general insert
            const HeaderIndex* idx = add_to_index(hs[i], hashes[i], prev, &proofs[i], &batch);
            consider_new_header(idx);
            r.ok = true;
            r.index = prev = idx;
            batch.push_back(idx);
            ++i;
            continue;
        }
        r.ok = false;
        break;
    }
    out.resize(std::min(n, i + 1));  // up to and including the first failure
    return out;
}

// Full recompute (after invalidate / reconsider): one pass in height order marks every
// descendant of a failed header bad, then the most-work good header becomes the tip. O(n).
void HeaderChain::update_active_chain() {
    // in arrival order, so among equal-work tips the first one received wins (nSequenceId)
    std::vector<const HeaderIndex*> nodes;
    nodes.reserve(storage_.size());
    storage_.for_each([&](const HeaderIndex* e) { nodes.push_back(e); });
    std::stable_sort(nodes.begin(), nodes.end(),
                     [](const HeaderIndex* a, const HeaderIndex* b) { return a->height < b->height; });
    std::unordered_set<const HeaderIndex*> bad;
    const HeaderIndex* best = genesis_;
    for (const HeaderIndex* c : nodes) {
        if (failed_.count(c) || (c->prev && bad.count(c->prev))) {
            bad.insert(c);
            continue;
        }
        if (c->chain_work > best->chain_work) best = c;
    }
    set_active_tip(best);
}

// Re-point the active chain at `best`: only the entries from the fork point up change.
void HeaderChain::set_active_tip(const HeaderIndex* best) {
    ++version_;
    const size_t want = size_t(best->height) + 1;
    if (want > active_.capacity()) {
        // headroom for the next 2^20 headers (~35 days of chain): a 10k-header batch at height
        // 2.88M must not reallocate and copy a 23 MB vector (3 ms, profiles/README r6g)
        active_.reserve(want + (size_t(1) << 20));
    }
    active_.resize(want, nullptr);
    for (const HeaderIndex* p = best; p && active_[size_t(p->height)] != p; p = p->prev)
        active_[size_t(p->height)] = p;
}

// Incremental tip update after adding `idx` (ActivateBestChain for headers): a header with
// more work than the tip becomes the tip unless a header between it and the active chain
// failed. Costs the fork depth, not the chain length.
void HeaderChain::consider_new_header(const HeaderIndex* idx) {
    const HeaderIndex* t = active_.empty() ? genesis_ : active_.back();
    if (!(idx->chain_work > t->chain_work)) return;
    for (const HeaderIndex* p = idx; p; p = p->prev) {
        if (size_t(p->height) < active_.size() && active_[size_t(p->height)] == p) break;  // fork point
        if (failed_.count(p)) return;
    }
    set_active_tip(idx);
}

const HeaderIndex* HeaderChain::add_anchor(const std::vector<BlockHeader>& hs, int base_height,
                                           const ArithU256& base_work) {
    std::lock_guard<std::recursive_mutex> g(mu_);
    if (hs.empty() || base_height <= 0) throw std::invalid_argument("add_anchor: empty run or height <= 0");
    const HeaderIndex* prev = nullptr;
    ArithU256 work = base_work;
    for (size_t i = 0; i < hs.size(); ++i) {
        const BlockHeader& h = hs[i];
        const Uint256 hash = verifier_->block_hash(h, params_);
        if (prev != nullptr && h.prev != prev->hash) throw std::invalid_argument("add_anchor: headers do not link");
        if (index_.find(hash) != nullptr) throw std::invalid_argument("add_anchor: header already indexed");
        HeaderIndex& idx = *storage_.alloc();
        idx.hash = hash;
        idx.prev = prev;
        idx.height = base_height + int(i);
        idx.time = h.time;
        idx.bits = h.bits;
        idx.header = h;
        work = work + block_proof(h.bits);
        idx.chain_work = work;
        idx.skip = prev ? prev->ancestor(skip_height(idx.height)) : nullptr;
        index_.insert(&idx);
        prev = &idx;
    }
    ++version_;
    consider_new_header(prev);
    return prev;
}

const HeaderIndex* HeaderChain::tip() const {
    std::lock_guard<std::recursive_mutex> g(mu_);
    return active_.empty() ? nullptr : active_.back();
}

const HeaderIndex* HeaderChain::at_height(int h) const {
    std::lock_guard<std::recursive_mutex> g(mu_);
    if (h < 0 || size_t(h) >= active_.size()) return nullptr;
    return active_[size_t(h)];
}

const HeaderIndex* HeaderChain::find(const Uint256& hash) const {
    std::lock_guard<std::recursive_mutex> g(mu_);
    return index_.find(hash);
}

void HeaderChain::invalidate(const Uint256& hash) {
    std::lock_guard<std::recursive_mutex> g(mu_);
    const HeaderIndex* e = index_.find(hash);
    if (e == nullptr || e == genesis_) return;
    failed_[e] = true;
    ++version_;
    update_active_chain();
}

void HeaderChain::reconsider(const Uint256& hash) {
    std::lock_guard<std::recursive_mutex> g(mu_);
    const HeaderIndex* node = index_.find(hash);
    if (node == nullptr) return;
    // ResetBlockFailureFlags: the block, its descendants and its ancestors become valid again
    auto walk = [](const HeaderIndex* x, int height) {
        while (x && x->height > height) x = x->prev;
        return x;
    };
    for (auto f = failed_.begin(); f != failed_.end();) {
        const HeaderIndex* x = f->first;
        const bool related = x->height >= node->height ? walk(x, node->height) == node : walk(node, x->height) == x;
        f = related ? failed_.erase(f) : std::next(f);
    }
    ++version_;
    update_active_chain();
}

// ---------------------------------------------------------------- block files
BlockStore::BlockStore(std::string dir, const u8 magic[4], u32 act) : dir_(std::move(dir)), act_(act) {
    std::memcpy(magic_, magic, 4);
    ::mkdir(dir_.c_str(), 0755);
    // continue after the highest-numbered blk file (pruning leaves gaps below it)
    file_ = -1;
    if (DIR* d = ::opendir(dir_.c_str())) {
        while (dirent* e = ::readdir(d)) {
            int n = -1;
            char tail = 0;
            if (std::sscanf(e->d_name, "blk%5d.dat%c", &n, &tail) == 1 && n >= 0 && std::strlen(e->d_name) == 12)
                file_ = std::max(file_, n);
        }
        ::closedir(d);
    }
    if (file_ < 0) {
        file_ = 0;
        return;
    }
    struct stat st;
    if (::stat(path(file_).c_str(), &st) == 0) file_size_ = u32(st.st_size);
}

std::string BlockStore::path(int file) const {
    char name[32];
    std::snprintf(name, sizeof(name), "/blk%05d.dat", file);
    return dir_ + name;
}

BlockStore::Pos BlockStore::write(const Block& b) { return write_raw(b.bytes(act_, true)); }

BlockStore::Pos BlockStore::write_raw(const Bytes& data) {
    std::lock_guard<std::mutex> g(mu_);
    const u32 rec = u32(data.size()) + 8;
    if (file_size_ > 0 && file_size_ + rec > max_file_) {
        ++file_;
        file_size_ = 0;
    }
    FILE* f = std::fopen(path(file_).c_str(), "ab");
    if (!f) throw std::runtime_error("cannot open " + path(file_));
    u8 hdr[8];
    std::memcpy(hdr, magic_, 4);
    store_le32(hdr + 4, u32(data.size()));
    const bool ok = std::fwrite(hdr, 1, 8, f) == 8 && std::fwrite(data.data(), 1, data.size(), f) == data.size();
    std::fflush(f);
    std::fclose(f);
    if (!ok) throw std::runtime_error("short write to " + path(file_));
    Pos p;
    p.file = file_;
    p.offset = file_size_ + 8;
    p.size = u32(data.size());
    file_size_ += rec;
    return p;
}

Bytes BlockStore::read_raw(const Pos& pos) const {
    FILE* f = std::fopen(path(pos.file).c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open " + path(pos.file));
    Bytes hdr(8), data(pos.size);
    bool ok = std::fseek(f, long(pos.offset) - 8, SEEK_SET) == 0 && std::fread(hdr.data(), 1, 8, f) == 8;
    ok = ok && std::memcmp(hdr.data(), magic_, 4) == 0 && load_le32(hdr.data() + 4) == pos.size;
    ok = ok && std::fread(data.data(), 1, data.size(), f) == data.size();
    std::fclose(f);
    if (!ok) throw std::runtime_error("ReadBlockFromDisk: bad record");
    return data;
}

Block BlockStore::read(const Pos& pos) const {
    Bytes d = read_raw(pos);
    Reader r(d);
    return Block::deserialize(r, act_);
}

std::vector<std::pair<BlockStore::Pos, Bytes>> BlockStore::scan() const {
    std::vector<std::pair<Pos, Bytes>> out;
    for (int file = 0; file <= file_; ++file) {
        FILE* f = std::fopen(path(file).c_str(), "rb");
        if (!f) continue;  // a pruned file
        u32 off = 0;
        for (;;) {
            u8 hdr[8];
            if (std::fread(hdr, 1, 8, f) != 8) break;
            if (std::memcmp(hdr, magic_, 4) != 0) break;
            const u32 size = load_le32(hdr + 4);
            Bytes d(size);
            if (std::fread(d.data(), 1, size, f) != size) break;
            Pos p{file, off + 8, size};
            out.emplace_back(p, std::move(d));
            off += 8 + size;
        }
        std::fclose(f);
    }
    return out;
}

}  // namespace nodexa
