// Header chain (block index + active chain) and blk?????.dat block files.
//
// Parity: CBlockIndex / CChain (src/chain.h:172,465), AcceptBlockHeader /
// ProcessNewBlockHeaders (src/validation.cpp:11957-12035), CheckBlockHeader
// (:11638-11665, checkpoint-gated mix-only vs full KawPow), ContextualCheck-
// BlockHeader (:11811-11875: bad-diffbits, checkpoint forks, time-too-old
// (MTP), time-too-new (2 h, 12 min once DGW is active), asset block version),
// WriteBlockToDisk / ReadBlockFromDisk framing (src/validation.cpp:1275-1328,
// sizes src/validation.h:89-93).
//
// Design: the PoW check is a pluggable verifier so the same pipeline runs
// with the CPU golden model, with GPU batch verification (headers pre-checked
// in bulk, then accepted with `check_pow=false`), or the mix-only fast path.
#pragma once

#include <deque>
#include <functional>
#include <memory>
#include <new>
#include <mutex>
#include <unordered_map>

#include "pow_rules.hpp"

namespace nodexa {

constexpr int64_t kMaxFutureBlockTime = 2 * 60 * 60;
constexpr int64_t kMaxFutureBlockTimeDgw = kMaxFutureBlockTime / 10;
constexpr int32_t kVersionBitsTopBitsAssets = 0x30000000;
constexpr u32 kMaxBlockfileSize = 0x8000000;  // 128 MiB

struct PowVerifier {
    virtual ~PowVerifier() = default;
    // CBlockHeader::GetHash (X16R / X16RV2 / KawPow mix-only).
    virtual Uint256 block_hash(const BlockHeader& h, const ChainParams& p) const = 0;
    // CBlockHeader::GetHashFull: (pow hash, computed mix_hash).
    virtual Uint256 block_hash_full(const BlockHeader& h, const ChainParams& p, Uint256& mix) const = 0;
};

// CPU golden verifier (KawPow light mode via cached epoch contexts, X16R CPU).
struct CpuPowVerifier : PowVerifier {
    Uint256 block_hash(const BlockHeader& h, const ChainParams& p) const override;
    Uint256 block_hash_full(const BlockHeader& h, const ChainParams& p, Uint256& mix) const override;
};

struct AcceptResult {
    bool ok = false;
    bool duplicate = false;
    std::string reject;  // reference reject reason ("high-hash", "bad-diffbits", ...)
    int dos = 0;
    const HeaderIndex* index = nullptr;
};

// Index entries live in fixed 1024-entry chunks: stable addresses, one allocation per chunk
// instead of one per header. A batch takes its entries' storage in one call and constructs them
// in parallel (the first touch of fresh pages is then spread over the cores too).
class HeaderArena {
public:
    static constexpr size_t kChunk = 1024;
    HeaderArena() = default;
    HeaderArena(const HeaderArena&) = delete;
    HeaderArena& operator=(const HeaderArena&) = delete;
    ~HeaderArena() {
        for (size_t i = 0; i < used_; ++i) at(i)->~HeaderIndex();
        for (void* c : chunks_) ::operator delete(c);
    }
    HeaderIndex* alloc() {
        HeaderIndex* e = nullptr;
        emplace_n(1, &e, [&] { new (e) HeaderIndex(); });
        return e;
    }
    // Storage for n entries (out[k]); `construct` placement-news every one of them (from any
    // number of threads). The entries count as allocated -- and are destroyed with the arena --
    // only once `construct` has returned, so a throw leaves nothing half-built behind.
    template <class F>
    void emplace_n(size_t n, HeaderIndex** out, F&& construct) {
        while (used_ + n > chunks_.size() * kChunk) chunks_.push_back(::operator new(kChunk * sizeof(HeaderIndex)));
        for (size_t k = 0; k < n; ++k) out[k] = at(used_ + k);
        construct();
        used_ += n;
    }
    size_t size() const { return used_; }
    template <class F>
    void for_each(F&& f) const {  // allocation order
        for (size_t i = 0; i < used_; ++i) f(at(i));
    }

private:
    HeaderIndex* at(size_t i) const { return static_cast<HeaderIndex*>(chunks_[i / kChunk]) + i % kChunk; }
    std::vector<void*> chunks_;
    size_t used_ = 0;
};

// The block index (mapBlockIndex): an open-addressing table of entries keyed by their own
// block hash. No per-entry allocation and one probe sequence per lookup; entries are never
// removed (an invalid header stays indexed and is marked failed). Lookups are safe from many
// threads while nothing inserts.
class HeaderHashTable {
public:
    HeaderIndex* find(const Uint256& h) const {
        if (slots_.empty()) return nullptr;
        for (size_t i = slot(h);; i = (i + 1) & mask_) {
            HeaderIndex* e = slots_[i];
            if (e == nullptr || e->hash == h) return e;
        }
    }
    void insert(HeaderIndex* e) {  // e->hash must not be present
        if ((n_ + 1) * 2 > slots_.size()) grow(std::max<size_t>(64, slots_.size() * 2));
        size_t i = slot(e->hash);
        while (slots_[i]) i = (i + 1) & mask_;
        slots_[i] = e;
        ++n_;
    }
    // Inserts from many threads at once into a table reserve()d for them (claims empty slots
    // with a compare-and-swap; nothing reads the table meanwhile). The caller adds the count.
    void insert_concurrent(HeaderIndex* e) {
        size_t i = slot(e->hash);
        for (;; i = (i + 1) & mask_) {
            HeaderIndex* expect = nullptr;
            if (__atomic_compare_exchange_n(&slots_[i], &expect, e, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) return;
        }
    }
    void add_count(size_t k) { n_ += k; }
    void reserve(size_t n) {
        size_t cap = 64;
        while (cap < 2 * n) cap *= 2;
        if (cap > slots_.size()) grow(cap);
    }
    size_t size() const { return n_; }
    template <class F>
    void for_each(F&& f) const {
        for (HeaderIndex* e : slots_)
            if (e) f(e);
    }

private:
    size_t slot(const Uint256& h) const {
        u64 x;
        std::memcpy(&x, h.data, 8);
        return size_t((x * 0x9E3779B97F4A7C15ull) >> shift_);
    }
    void grow(size_t cap) {
        std::vector<HeaderIndex*> old;
        old.swap(slots_);
        slots_.assign(cap, nullptr);
        mask_ = cap - 1;
        shift_ = 64 - unsigned(__builtin_ctzll(cap));
        n_ = 0;
        for (HeaderIndex* e : old)
            if (e) insert(e);
    }
    std::vector<HeaderIndex*> slots_;
    size_t n_ = 0, mask_ = 0;
    unsigned shift_ = 64;
};

// accept_headers in two phases (HeaderChain::prepare_headers / commit_headers): the context-free
// and read-only per-header work of a batch -- hashes, block proofs, parent MTPs, expected nBits,
// contextual rules, freshness -- then the serial index insert. The resident batch verify
// (models/verify.py) prepares while the device is still finishing the PoW verdicts and commits
// the verified prefix afterwards; the commit redoes everything when the index changed between.
struct AcceptPrep {
    const BlockHeader* hs = nullptr;
    size_t n = 0;
    int64_t adjusted_time = 0;
    bool check_pow = false;
    std::vector<Uint256> hashes;
    std::vector<u32> expected;
    std::vector<u8> have, have_mtp;
    std::vector<ArithU256> proofs;
    std::vector<int64_t> mtp;
    std::vector<AcceptResult> pre;
    std::vector<u8> ctx, fresh;  // empty: the batch takes the header-by-header path
    int base_height = 0;
    u64 version = 0;  // the chain's version when prepared
    bool strict_height = false;
    std::vector<u32> known_bits;  // the caller's nBits (0 = unknown), kept for a re-prepare
};

class HeaderChain {
public:
    HeaderChain(ChainParams params, std::shared_ptr<const PowVerifier> verifier);

    const ChainParams& params() const { return params_; }
    ChainParams& mutable_params() { return params_; }
    const PowVerifier& verifier() const { return *verifier_; }

    // CheckBlockHeader (context-free PoW check).
    AcceptResult check_header(const BlockHeader& h, bool check_pow) const;
    AcceptResult accept_header(const BlockHeader& h, int64_t adjusted_time, bool check_pow = true);
    // Accepts headers in order; stops at the first failure (ProcessNewBlockHeaders).
    // `known_hashes` (one per header, storage order): block hashes the caller already has (the
    // batch PoW stage computes them), so the host does not hash the batch again.
    // `known_bits` (one per header, 0 = unknown): the DGW nBits of each header, computed by the
    // caller from dgw_series (the GPU batch kernel hip/kernels/dgw.hip).
    std::vector<AcceptResult> accept_headers(const std::vector<BlockHeader>& hs, int64_t adjusted_time,
                                             bool check_pow = true, const std::vector<Uint256>* known_hashes = nullptr,
                                             const std::vector<u32>* known_bits = nullptr);
    // The (nTime, nBits) series DarkGravityWave reads for a batch that extends a known header
    // linearly: up to 180 ancestors of the batch's parent (oldest first, `a` of them) then the
    // batch. False if the batch is not linear or the network does not retarget with DGW.
    bool dgw_series(const std::vector<BlockHeader>& hs, const std::vector<Uint256>& hashes, std::vector<u32>& times,
                    std::vector<u32>& bits, size_t& a, int& base_height) const {
        return dgw_series(hs.data(), hs.size(), hashes.data(), times, bits, a, base_height);
    }
    // The same over a contiguous range of headers (a HeaderBatch's own storage: no copies).
    bool dgw_series(const BlockHeader* hs, size_t n, const Uint256* hashes, std::vector<u32>& times,
                    std::vector<u32>& bits, size_t& a, int& base_height) const;
    std::vector<AcceptResult> accept_headers(const BlockHeader* hs, size_t n, int64_t adjusted_time, bool check_pow,
                                             const Uint256* known_hashes, const u32* known_bits);
    // The two phases of accept_headers (AcceptPrep); commit accepts headers [0, hi) of the
    // prepared ones (a verified prefix), exactly as accept_headers over that prefix would.
    AcceptPrep prepare_headers(const BlockHeader* hs, size_t n, int64_t adjusted_time, bool check_pow,
                               const Uint256* known_hashes, const u32* known_bits) const;
    std::vector<AcceptResult> commit_headers(AcceptPrep& p, size_t hi);

    // A run of stored headers continuing from a point this index does not hold (the state a node
    // restored from its block-index database at height `base_height` has: LoadBlockIndexDB does
    // not re-validate stored entries either): hs[0] at `base_height`, each next header's prev the
    // previous one's hash, chain work `base_work` + the run's proofs. Not checked (trusted, like a
    // loaded index); enough of them (>= 180) make DarkGravityWave and the median time past of the
    // headers built on top exact. Returns the last entry (the new tip when it has the most work).
    const HeaderIndex* add_anchor(const std::vector<BlockHeader>& hs, int base_height, const ArithU256& base_work);

    const HeaderIndex* tip() const;
    const HeaderIndex* genesis() const { return genesis_; }
    const HeaderIndex* at_height(int h) const;
    const HeaderIndex* find(const Uint256& hash) const;
    int height() const { const HeaderIndex* t = tip(); return t ? t->height : -1; }
    bool in_active_chain(const HeaderIndex* idx) const { return idx && at_height(idx->height) == idx; }
    size_t size() const { return index_.size(); }
    // Marks a block (and descendants) invalid and re-selects the tip (invalidateblock).
    void invalidate(const Uint256& hash);
    void reconsider(const Uint256& hash);
    u32 next_bits(const BlockHeader& candidate) const;  // GetNextWorkRequired on the tip
    bool strict_kawpow_height = false;  // policy: header nHeight must equal index height
    // -maxreorg guard (ContextualCheckBlockHeader, src/validation.cpp:11815-11827): > 0 rejects a
    // header whose parent is this many or more blocks below the active tip. The node arms it
    // only while it has >= -minreorgpeers peers and a tip younger than -minreorgage.
    int max_reorg_depth = 0;

    static constexpr size_t kParallelAcceptMin = 64;  // batch size from which accept_headers precomputes

private:
    AcceptResult accept_header_impl(const BlockHeader& h, const Uint256* known_hash, int64_t adjusted_time,
                                    bool check_pow, const u32* expected_bits, const AcceptResult* precheck, const ArithU256* proof = nullptr,
                                    const int64_t* prev_mtp = nullptr);
    // `batch`: the entries a linear batch added so far (batch[k] at height batch[0]->height + k)
    const HeaderIndex* add_to_index(const BlockHeader& h, const Uint256& hash, const HeaderIndex* prev,
                                    const ArithU256* proof = nullptr,
                                    const std::vector<const HeaderIndex*>* batch = nullptr);
    bool contextual_rules(const BlockHeader& h, const Uint256& hash, int height, u32 expected_bits, int64_t prev_mtp,
                          int64_t adjusted_time, bool cp_fork, AcceptResult& r) const;
    void update_active_chain();
    void set_active_tip(const HeaderIndex* best);
    void consider_new_header(const HeaderIndex* idx);

    ChainParams params_;
    std::shared_ptr<const PowVerifier> verifier_;
    mutable std::recursive_mutex mu_;
    HeaderArena storage_;
    HeaderHashTable index_;
    std::unordered_map<const HeaderIndex*, bool> failed_;
    std::vector<const HeaderIndex*> active_;
    const HeaderIndex* genesis_ = nullptr;
    u64 version_ = 0;  // bumped by every change of the index, the failed set or the active chain
};

// blk?????.dat files: [magic 4][u32 size][block] records, 128 MiB per file.
class BlockStore {
public:
    BlockStore(std::string dir, const u8 magic[4], u32 kawpow_activation_time);
    struct Pos { int file = -1; u32 offset = 0; u32 size = 0; };
    Pos write(const Block& b);
    Pos write_raw(const Bytes& serialized_block);
    Bytes read_raw(const Pos& pos) const;
    Block read(const Pos& pos) const;
    // Scan every record of every blk file (reindex / -loadblock). Stops on a bad magic.
    std::vector<std::pair<Pos, Bytes>> scan() const;
    std::string path(int file) const;
    int current_file() const { return file_; }
    // files roll over past this size (MAX_BLOCKFILE_SIZE; smaller only to exercise pruning)
    void set_max_file_size(u32 n) { max_file_ = n; }

private:
    std::string dir_;
    u8 magic_[4];
    u32 act_;
    int file_ = 0;
    u32 file_size_ = 0;
    u32 max_file_ = kMaxBlockfileSize;
    mutable std::mutex mu_;
};

}  // namespace nodexa
