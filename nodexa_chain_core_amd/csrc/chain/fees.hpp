// Block-confirmation fee estimator.
//
// Parity (behaviour): CBlockPolicyEstimator / TxConfirmStats (src/policy/fees.h:80-306,
// src/policy/fees.cpp:77-1037): feerate buckets 1000..1e7 sat/kB spaced by 1.05 plus an
// infinite bucket; three horizons (short 12 x 1 block decay .962, medium 24 x 2 decay .9952,
// long 42 x 24 decay .99931); per horizon exponentially decayed confirmed / failed / total
// counts and feerate sums per bucket plus a ring of still-unconfirmed pool entries by entry
// height; estimateRawFee, estimateCombinedFee, estimateConservativeFee and estimateSmartFee
// (60 % at target/2, 85 % at target, 95 % at 2x target, conservative = every longer horizon
// too); fee_estimates.dat in the reference's serialization (version 149900, CLIENT_VERSION
// 4040402), so a file written by clore_blockchaind loads here and back.
//
// Layout: each horizon keeps its counters as flat bucket-minor arrays (one row per
// confirmation period), so a decay pass or a bucket-range scan walks contiguous doubles.
#pragma once

#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "serialize.hpp"
#include "uint256.hpp"

namespace nodexa {

enum class FeeHorizon { Short = 0, Medium = 1, Long = 2 };
enum class FeeReason { None = 0, HalfEstimate, FullEstimate, DoubleEstimate, Conservative };

struct FeeBucketRange {   // EstimatorBucket
    double start = -1, end = -1;
    double within_target = 0, total_confirmed = 0, in_mempool = 0, left_mempool = 0;
};

struct FeeEstimation {    // EstimationResult
    FeeBucketRange pass, fail;
    double decay = 0;
    unsigned scale = 0;
};

// One time horizon of confirmation history (TxConfirmStats).
class ConfirmHistory {
public:
    ConfirmHistory(const std::vector<double>* bounds, unsigned periods, double decay, unsigned scale);

    unsigned max_confirms() const { return scale_ * periods_; }
    double decay() const { return decay_; }
    unsigned scale() const { return scale_; }

    void roll(u32 height);                                   // ClearCurrent
    void decay_all();                                        // UpdateMovingAverages
    void record(int blocks_to_confirm, unsigned bucket, double feerate);
    void add_unconfirmed(u32 height, unsigned bucket);       // NewTx
    void remove(u32 entry_height, u32 best_seen, unsigned bucket, bool in_block);
    // EstimateMedianVal with requireGreater = true; -1 when no bucket range passes.
    double median(int target, double sufficient, double success, u32 height, FeeEstimation* out) const;

    void write(Writer& w) const;
    void read(Reader& r, size_t nbuckets);   // throws std::runtime_error on a corrupt file

private:
    double& conf(unsigned period, unsigned b) { return conf_[size_t(period) * nb_ + b]; }
    double& fail(unsigned period, unsigned b) { return fail_[size_t(period) * nb_ + b]; }
    double conf(unsigned period, unsigned b) const { return conf_[size_t(period) * nb_ + b]; }
    double fail(unsigned period, unsigned b) const { return fail_[size_t(period) * nb_ + b]; }
    void size_unconfirmed();

    const std::vector<double>* bounds_;
    size_t nb_;
    unsigned periods_;
    double decay_;
    unsigned scale_;
    std::vector<double> conf_, fail_;   // [period][bucket]
    std::vector<double> count_, sum_;   // [bucket]
    std::vector<int> unconf_;           // [max_confirms ring slot][bucket]
    std::vector<int> old_unconf_;       // [bucket]
};

class FeeEstimator {
public:
    static constexpr int kFileVersion = 149900;
    static constexpr int kClientVersion = 4040402;

    FeeEstimator();

    // processTransaction: a pool entry admitted at chain height `height` (valid = the node is
    // current, the tx is not a replacement and has no in-pool parents).
    void process_tx(const Uint256& txid, u32 height, int64_t fee, int64_t vsize, bool valid);
    // processBlock: the pool entries a block at `height` confirmed.
    void process_block(u32 height, const std::vector<Uint256>& txids);
    bool remove_tx(const Uint256& txid, bool in_block);
    void flush_unconfirmed();   // FlushUnconfirmed: every tracked entry counts as a failure

    int64_t estimate_fee(int target) const;   // sat/kB, 0 = no estimate
    int64_t estimate_raw_fee(int target, double threshold, FeeHorizon h, FeeEstimation* out) const;
    int64_t estimate_smart_fee(int target, bool conservative, int* returned_target, FeeReason* reason,
                               FeeEstimation* out) const;
    unsigned highest_target_tracked(FeeHorizon h) const;
    unsigned max_usable_estimate() const;

    Bytes serialize() const;
    bool deserialize(const Bytes& b, std::string* err);

    size_t tracked() const;
    u32 best_seen_height() const { return best_seen_; }

private:
    struct Tracked { u32 height; unsigned bucket; double feerate; };
    unsigned bucket_of(double feerate) const;
    const ConfirmHistory& horizon(FeeHorizon h) const;
    bool remove_locked(const Uint256& txid, bool in_block);
    unsigned block_span() const;
    unsigned historical_span() const;
    double combined(unsigned target, double success, bool check_shorter, FeeEstimation* out) const;
    double conservative(unsigned double_target, FeeEstimation* out) const;

    mutable std::mutex mu_;
    std::vector<double> bounds_;
    ConfirmHistory med_, short_, long_;
    std::unordered_map<Uint256, Tracked, Uint256Hasher> pool_;
    u32 best_seen_ = 0, first_recorded_ = 0, hist_first_ = 0, hist_best_ = 0;
};

const char* fee_reason_string(FeeReason r);

}  // namespace nodexa
