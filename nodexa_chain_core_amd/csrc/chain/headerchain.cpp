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
                                              const ArithU256* proof) {
    storage_.emplace_back();
    HeaderIndex& idx = storage_.back();
    idx.hash = hash;
    idx.prev = prev;
    idx.height = prev ? prev->height + 1 : 0;
    idx.time = h.time;
    idx.bits = h.bits;
    idx.header = h;
    idx.chain_work = (prev ? prev->chain_work : ArithU256()) + (proof ? *proof : block_proof(h.bits));
    if (prev) {
        // skip pointer: GetSkipHeight (src/chain.cpp)
        auto invert_low = [](int n) { return n & (n - 1); };
        const int hgt = idx.height;
        const int skip_h = hgt < 2 ? 0 : ((hgt & 1) ? invert_low(invert_low(hgt - 1)) + 1 : invert_low(hgt));
        idx.skip = prev->ancestor(skip_h);
    }
    index_[hash] = &idx;
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
    auto self = index_.find(hash);
    if (self != index_.end()) {
        r.index = self->second;
        r.duplicate = true;
        if (failed_.count(self->second)) {
            r.reject = "duplicate";
            return r;
        }
        r.ok = true;
        return r;
    }
    r = precheck ? *precheck : check_header(h, check_pow);
    if (!r.ok) return r;
    r.ok = false;
    auto pit = index_.find(h.prev);
    if (pit == index_.end()) {
        r.reject = "prev-blk-not-found";
        r.dos = 10;
        return r;
    }
    const HeaderIndex* prev = pit->second;
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
    if (h.bits != (expected_bits ? *expected_bits : next_work_required(prev, h, params_))) {
        r.reject = "bad-diffbits";
        r.dos = 100;
        return r;
    }
    const int cp = params_.last_checkpoint_height();
    if (cp >= 0 && height < cp && at_height(cp) != nullptr) {
        r.reject = "bad-fork-prior-to-checkpoint";
        r.dos = 100;
        return r;
    }
    auto cpit = params_.checkpoints.find(height);
    if (cpit != params_.checkpoints.end() && cpit->second != hash) {
        r.reject = "checkpoint mismatch";
        r.dos = 100;
        return r;
    }
    if (int64_t(h.time) <= (prev_mtp ? *prev_mtp : prev->median_time_past())) {
        r.reject = "time-too-old";
        return r;
    }
    const int64_t max_future = (height >= params_.dgw_activation_block) ? kMaxFutureBlockTimeDgw : kMaxFutureBlockTime;
    if (int64_t(h.time) > adjusted_time + max_future) {
        r.reject = "time-too-new";
        return r;
    }
    if (h.version < kVersionBitsTopBitsAssets) {
        char buf[48];
        std::snprintf(buf, sizeof(buf), "bad-version(0x%08x)", unsigned(h.version));
        r.reject = buf;
        return r;
    }
    // Equihash extension era (new): the flag bit is required from the activation
    // time on and forbidden before it (so reference-network headers never parse
    // as extended ones), and the extended header commits to its height.
    const bool eq_era = h.time >= params_.equihash_activation_time;
    if (eq_era != h.is_equihash()) {
        r.reject = eq_era ? "bad-version(equihash-required)" : "bad-version(equihash-not-active)";
        r.dos = 100;
        return r;
    }
    if (h.is_equihash() && int(h.height) != height) {
        r.reject = "bad-height";
        r.dos = 100;
        return r;
    }
    // The reference never checks that a KawPow header's nHeight equals its index
    // height (the epoch/period therefore follow the claimed height). Off by
    // default for consensus compatibility; -strictheight turns it on as policy.
    if (strict_kawpow_height && params_.algo_for(h.time) == PowAlgo::KAWPOW && int(h.height) != height) {
        r.reject = "bad-height";
        r.dos = 100;
        return r;
    }
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
    auto pit = index_.find(hs[0].prev);
    bool linear = pit != index_.end();
    for (size_t i = 1; linear && i < n; ++i) linear = hs[i].prev == hashes[i - 1];
    const ConsensusParams& c = params_.consensus;
    if (!linear || (c.pow_allow_min_difficulty_blocks && c.pow_no_retargeting)) return false;
    const HeaderIndex* base = pit->second;
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

std::vector<AcceptResult> HeaderChain::accept_headers(const BlockHeader* hs, size_t n, int64_t adjusted_time,
                                                      bool check_pow, const Uint256* known_hashes,
                                                      const u32* known_bits) {
    std::lock_guard<std::recursive_mutex> g(mu_);
    std::vector<AcceptResult> out;
    out.reserve(n);
    std::vector<Uint256> hashes;
    std::vector<u32> expected;
    std::vector<u8> have(n, 0), have_mtp(n, 0);
    std::vector<ArithU256> proofs;
    std::vector<int64_t> mtp;
    std::vector<AcceptResult> pre;
    if (n >= kParallelAcceptMin && check_pow) {  // CheckBlockHeader (full PoW) is context-free
        pre.resize(n);
        parallel_for(n, [&](size_t i) { pre[i] = check_header(hs[i], true); });
    }
    if (n >= kParallelAcceptMin) {
        if (known_hashes) {
            hashes.assign(known_hashes, known_hashes + n);
        } else {
            hashes.resize(n);
            parallel_for(n, [&](size_t i) { hashes[i] = verifier_->block_hash(hs[i], params_); });
        }
        // context-free per-header work of the serial pass, done up front on all cores: the block
        // proof (2^256 / (target + 1), a 256-bit division) and, for a linear batch, the median
        // time past of each header's parent from the batch's own time series
        proofs.resize(n);
        parallel_for(n, [&](size_t i) { proofs[i] = block_proof(hs[i].bits); });
        std::vector<u32> times, bits;
        size_t a = 0;
        int base_height = 0;
        if (dgw_series(hs, n, hashes.data(), times, bits, a, base_height)) {
            const bool from_genesis = a == size_t(base_height) + 1;  // the series reaches genesis
            mtp.resize(n);
            parallel_for(n, [&](size_t i) {
                const int64_t j = int64_t(a) - 1 + int64_t(i);  // series index of header i's parent
                if (j < 10 && !from_genesis) return;
                int64_t w[11];
                int m = 0;
                for (int64_t k = j; k >= 0 && m < 11; --k) w[m++] = times[size_t(k)];
                std::sort(w, w + m);
                mtp[i] = w[m / 2];
                have_mtp[i] = 1;
            });
            if (known_bits) {
                // computed by the caller from the same series (the GPU batch kernel, dgw.hip);
                // 0 = not a DGW header, left to the serial path
                expected.assign(known_bits, known_bits + n);
                for (size_t i = 0; i < n; ++i) have[i] = expected[i] != 0;
            } else {
                const u32 limit_compact = ArithU256::from_uint256(params_.consensus.pow_limit).get_compact();
                expected.resize(n);
                parallel_for(n, [&](size_t i) {
                    const int last_height = base_height + int(i);  // height of header i's parent
                    if (last_height + 1 < params_.dgw_activation_block) return;  // BTC retarget: serial path
                    expected[i] = last_height < kDgwPastBlocks
                                      ? limit_compact
                                      : dgw_average(times.data(), bits.data(), int64_t(a) - 1 + int64_t(i), hs[i].time,
                                                    params_);
                    have[i] = 1;
                });
            }
        }
    }
    for (size_t i = 0; i < n; ++i) {
        out.push_back(accept_header_impl(hs[i], hashes.empty() ? nullptr : &hashes[i], adjusted_time, check_pow,
                                         have[i] ? &expected[i] : nullptr, pre.empty() ? nullptr : &pre[i],
                                         proofs.empty() ? nullptr : &proofs[i], have_mtp[i] ? &mtp[i] : nullptr));
        if (!out.back().ok) break;
    }
    return out;
}

// Full recompute (after invalidate / reconsider): one pass in height order marks every
// descendant of a failed header bad, then the most-work good header becomes the tip. O(n).
void HeaderChain::update_active_chain() {
    std::vector<const HeaderIndex*> nodes;
    nodes.reserve(index_.size());
    for (auto& kv : index_) nodes.push_back(kv.second);
    std::sort(nodes.begin(), nodes.end(),
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
    active_.resize(size_t(best->height) + 1, nullptr);
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
    auto it = index_.find(hash);
    return it == index_.end() ? nullptr : it->second;
}

void HeaderChain::invalidate(const Uint256& hash) {
    std::lock_guard<std::recursive_mutex> g(mu_);
    auto it = index_.find(hash);
    if (it == index_.end() || it->second == genesis_) return;
    failed_[it->second] = true;
    update_active_chain();
}

void HeaderChain::reconsider(const Uint256& hash) {
    std::lock_guard<std::recursive_mutex> g(mu_);
    auto it = index_.find(hash);
    if (it == index_.end()) return;
    // ResetBlockFailureFlags: the block, its descendants and its ancestors become valid again
    const HeaderIndex* node = it->second;
    auto walk = [](const HeaderIndex* x, int height) {
        while (x && x->height > height) x = x->prev;
        return x;
    };
    for (auto f = failed_.begin(); f != failed_.end();) {
        const HeaderIndex* x = f->first;
        const bool related = x->height >= node->height ? walk(x, node->height) == node : walk(node, x->height) == x;
        f = related ? failed_.erase(f) : std::next(f);
    }
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
