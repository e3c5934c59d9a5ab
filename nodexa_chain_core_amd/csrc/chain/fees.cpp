// Block-confirmation fee estimator. See fees.hpp for the parity map
// (src/policy/fees.cpp:77-1037).
#include "fees.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>

namespace nodexa {

namespace {

constexpr double kInfFeerate = 1e99;
constexpr double kMinBucket = 1000, kMaxBucket = 1e7, kSpacing = 1.05;   // src/policy/fees.h:182-190
constexpr unsigned kShortPeriods = 12, kShortScale = 1;
constexpr unsigned kMedPeriods = 24, kMedScale = 2;
constexpr unsigned kLongPeriods = 42, kLongScale = 24;
constexpr double kShortDecay = .962, kMedDecay = .9952, kLongDecay = .99931;
constexpr double kHalfSuccess = .6, kSuccess = .85, kDoubleSuccess = .95;
constexpr double kSufficientFeeTxs = 0.1, kSufficientTxsShort = 0.5;
constexpr unsigned kOldestHistory = 6 * 1008;

void put_double(Writer& w, double d) { u64 v; std::memcpy(&v, &d, 8); w.u64_(v); }
double get_double(Reader& r) { u64 v = r.u64_(); double d; std::memcpy(&d, &v, 8); return d; }

void put_vec(Writer& w, const double* p, size_t n) {
    w.compact_size(n);
    for (size_t i = 0; i < n; ++i) put_double(w, p[i]);
}
std::vector<double> get_vec(Reader& r) {
    const u64 n = r.compact_size();
    std::vector<double> v;
    v.reserve(size_t(n));
    for (u64 i = 0; i < n; ++i) v.push_back(get_double(r));
    return v;
}

std::vector<double> make_bounds() {
    std::vector<double> b;
    for (double x = kMinBucket; x <= kMaxBucket; x *= kSpacing) b.push_back(x);
    b.push_back(kInfFeerate);
    return b;
}

}  // namespace

const char* fee_reason_string(FeeReason r) {   // StringForFeeReason
    switch (r) {
    case FeeReason::None: return "None";
    case FeeReason::HalfEstimate: return "Half Target 60% Threshold";
    case FeeReason::FullEstimate: return "Target 85% Threshold";
    case FeeReason::DoubleEstimate: return "Double Target 95% Threshold";
    case FeeReason::Conservative: return "Conservative Double Target longer horizon";
    }
    return "Unknown";
}

// ---------------------------------------------------------------- ConfirmHistory

ConfirmHistory::ConfirmHistory(const std::vector<double>* bounds, unsigned periods, double decay, unsigned scale)
    : bounds_(bounds), nb_(bounds->size()), periods_(periods), decay_(decay), scale_(scale) {
    if (scale == 0) throw std::invalid_argument("ConfirmHistory: scale must be non-zero");
    conf_.assign(size_t(periods_) * nb_, 0.0);
    fail_.assign(size_t(periods_) * nb_, 0.0);
    count_.assign(nb_, 0.0);
    sum_.assign(nb_, 0.0);
    size_unconfirmed();
}

void ConfirmHistory::size_unconfirmed() {
    unconf_.assign(size_t(max_confirms()) * nb_, 0);
    old_unconf_.assign(nb_, 0);
}

void ConfirmHistory::roll(u32 height) {
    int* slot = &unconf_[size_t(height % max_confirms()) * nb_];
    for (size_t b = 0; b < nb_; ++b) {
        old_unconf_[b] += slot[b];
        slot[b] = 0;
    }
}

void ConfirmHistory::decay_all() {
    for (double& x : conf_) x *= decay_;
    for (double& x : fail_) x *= decay_;
    for (size_t b = 0; b < nb_; ++b) {
        sum_[b] *= decay_;
        count_[b] *= decay_;
    }
}

void ConfirmHistory::record(int blocks_to_confirm, unsigned bucket, double feerate) {
    if (blocks_to_confirm < 1) return;
    const unsigned first = unsigned((blocks_to_confirm + int(scale_) - 1) / int(scale_));
    for (unsigned p = first; p <= periods_; ++p) conf(p - 1, bucket) += 1;
    count_[bucket] += 1;
    sum_[bucket] += feerate;
}

void ConfirmHistory::add_unconfirmed(u32 height, unsigned bucket) {
    unconf_[size_t(height % max_confirms()) * nb_ + bucket] += 1;
}

void ConfirmHistory::remove(u32 entry_height, u32 best_seen, unsigned bucket, bool in_block) {
    int ago = int(best_seen - entry_height);
    if (best_seen == 0) ago = 0;
    if (ago < 0) return;   // cannot happen: entries never carry a height above the best seen
    if (ago >= int(max_confirms())) {
        if (old_unconf_[bucket] > 0) old_unconf_[bucket]--;
    } else {
        int& c = unconf_[size_t(entry_height % max_confirms()) * nb_ + bucket];
        if (c > 0) c--;
    }
    if (!in_block && unsigned(ago) >= scale_) {   // a failure only after a whole period unconfirmed
        const unsigned periods_ago = unsigned(ago) / scale_;
        for (unsigned p = 0; p < periods_ago && p < periods_; ++p) fail(p, bucket) += 1;
    }
}

double ConfirmHistory::median(int target, double sufficient, double success, u32 height, FeeEstimation* out) const {
    const std::vector<double>& bk = *bounds_;
    double n_conf = 0, total = 0, n_fail = 0;
    int extra = 0;
    const unsigned period = unsigned((target + int(scale_) - 1) / int(scale_));
    const int top = int(nb_) - 1;
    const u32 bins = max_confirms();
    unsigned cur_near = unsigned(top), best_near = unsigned(top), cur_far = unsigned(top), best_far = unsigned(top);
    bool found = false, new_range = true, passing = true;
    FeeBucketRange pass, failb;

    auto range_of = [&](unsigned a, unsigned c, FeeBucketRange& r) {
        const unsigned lo = std::min(a, c), hi = std::max(a, c);
        r.start = lo ? bk[lo - 1] : 0;
        r.end = bk[hi];
    };

    // from the highest feerate down: the lowest feerate whose whole upper range still passes
    for (int b = top; b >= 0; --b) {
        if (new_range) {
            cur_near = unsigned(b);
            new_range = false;
        }
        cur_far = unsigned(b);
        n_conf += conf(period - 1, unsigned(b));
        total += count_[size_t(b)];
        n_fail += fail(period - 1, unsigned(b));
        for (u32 k = u32(target); k < bins; ++k) extra += unconf_[size_t((height - k) % bins) * nb_ + size_t(b)];
        extra += old_unconf_[size_t(b)];
        if (total >= sufficient / (1 - decay_)) {
            const double pct = n_conf / (total + n_fail + extra);
            if (pct < success) {
                if (passing) {   // first failing range
                    range_of(cur_near, cur_far, failb);
                    failb.within_target = n_conf;
                    failb.total_confirmed = total;
                    failb.in_mempool = extra;
                    failb.left_mempool = n_fail;
                    passing = false;
                }
                continue;
            }
            failb = FeeBucketRange();
            found = true;
            passing = true;
            pass.within_target = n_conf;
            pass.total_confirmed = total;
            pass.in_mempool = extra;
            pass.left_mempool = n_fail;
            n_conf = total = n_fail = 0;
            extra = 0;
            best_near = cur_near;
            best_far = cur_far;
            new_range = true;
        }
    }

    double med = -1;
    const unsigned lo = std::min(best_near, best_far), hi = std::max(best_near, best_far);
    double tx_sum = 0;
    for (unsigned j = lo; j <= hi; ++j) tx_sum += count_[j];
    if (found && tx_sum != 0) {
        // average feerate of the bucket holding the median transaction of the passing range
        tx_sum /= 2;
        for (unsigned j = lo; j <= hi; ++j) {
            if (count_[j] < tx_sum) {
                tx_sum -= count_[j];
            } else {
                med = sum_[j] / count_[j];
                break;
            }
        }
        pass.start = lo ? bk[lo - 1] : 0;
        pass.end = bk[hi];
    }
    if (passing && !new_range) {   // trailing buckets without enough data count as the failure
        range_of(cur_near, cur_far, failb);
        failb.within_target = n_conf;
        failb.total_confirmed = total;
        failb.in_mempool = extra;
        failb.left_mempool = n_fail;
    }
    if (out) {
        out->pass = pass;
        out->fail = failb;
        out->decay = decay_;
        out->scale = scale_;
    }
    return med;
}

void ConfirmHistory::write(Writer& w) const {
    put_double(w, decay_);
    w.u32_(scale_);
    put_vec(w, sum_.data(), nb_);
    put_vec(w, count_.data(), nb_);
    w.compact_size(periods_);
    for (unsigned p = 0; p < periods_; ++p) put_vec(w, &conf_[size_t(p) * nb_], nb_);
    w.compact_size(periods_);
    for (unsigned p = 0; p < periods_; ++p) put_vec(w, &fail_[size_t(p) * nb_], nb_);
}

void ConfirmHistory::read(Reader& r, size_t nbuckets) {
    const double decay = get_double(r);
    if (!(decay > 0 && decay < 1)) throw std::runtime_error("Corrupt estimates file. Decay must be between 0 and 1 (non-inclusive)");
    const unsigned scale = r.u32_();
    if (scale == 0) throw std::runtime_error("Corrupt estimates file. Scale must be non-zero");
    std::vector<double> sum = get_vec(r);
    if (sum.size() != nbuckets) throw std::runtime_error("Corrupt estimates file. Mismatch in feerate average bucket count");
    std::vector<double> count = get_vec(r);
    if (count.size() != nbuckets) throw std::runtime_error("Corrupt estimates file. Mismatch in tx count bucket count");
    const u64 periods = r.compact_size();
    if (periods == 0 || periods * scale > 6 * 24 * 7)
        throw std::runtime_error("Corrupt estimates file.  Must maintain estimates for between 1 and 1008 (one week) confirms");
    std::vector<double> conf, fail;
    conf.reserve(size_t(periods) * nbuckets);
    for (u64 p = 0; p < periods; ++p) {
        std::vector<double> row = get_vec(r);
        if (row.size() != nbuckets) throw std::runtime_error("Corrupt estimates file. Mismatch in feerate conf average bucket count");
        conf.insert(conf.end(), row.begin(), row.end());
    }
    if (r.compact_size() != periods) throw std::runtime_error("Corrupt estimates file. Mismatch in confirms tracked for failures");
    fail.reserve(conf.size());
    for (u64 p = 0; p < periods; ++p) {
        std::vector<double> row = get_vec(r);
        if (row.size() != nbuckets) throw std::runtime_error("Corrupt estimates file. Mismatch in one of failure average bucket counts");
        fail.insert(fail.end(), row.begin(), row.end());
    }
    decay_ = decay;
    scale_ = scale;
    periods_ = unsigned(periods);
    nb_ = nbuckets;
    sum_ = std::move(sum);
    count_ = std::move(count);
    conf_ = std::move(conf);
    fail_ = std::move(fail);
    size_unconfirmed();
}

// ---------------------------------------------------------------- FeeEstimator

FeeEstimator::FeeEstimator()
    : bounds_(make_bounds()),
      med_(&bounds_, kMedPeriods, kMedDecay, kMedScale),
      short_(&bounds_, kShortPeriods, kShortDecay, kShortScale),
      long_(&bounds_, kLongPeriods, kLongDecay, kLongScale) {}

unsigned FeeEstimator::bucket_of(double feerate) const {   // bucketMap.lower_bound(val)
    return unsigned(std::lower_bound(bounds_.begin(), bounds_.end(), feerate) - bounds_.begin());
}

const ConfirmHistory& FeeEstimator::horizon(FeeHorizon h) const {
    switch (h) {
    case FeeHorizon::Short: return short_;
    case FeeHorizon::Medium: return med_;
    case FeeHorizon::Long: return long_;
    }
    throw std::out_of_range("unknown FeeEstimateHorizon");
}

void FeeEstimator::process_tx(const Uint256& txid, u32 height, int64_t fee, int64_t vsize, bool valid) {
    std::lock_guard<std::mutex> g(mu_);
    if (pool_.count(txid) || height != best_seen_ || !valid) return;   // side chains / not current
    const double feerate = double(vsize > 0 ? fee * 1000 / vsize : 0);  // CFeeRate(fee, size).GetFeePerK()
    const unsigned b = bucket_of(feerate);
    pool_[txid] = Tracked{height, b, feerate};
    med_.add_unconfirmed(height, b);
    short_.add_unconfirmed(height, b);
    long_.add_unconfirmed(height, b);
}

bool FeeEstimator::remove_locked(const Uint256& txid, bool in_block) {
    auto it = pool_.find(txid);
    if (it == pool_.end()) return false;
    const Tracked t = it->second;
    med_.remove(t.height, best_seen_, t.bucket, in_block);
    short_.remove(t.height, best_seen_, t.bucket, in_block);
    long_.remove(t.height, best_seen_, t.bucket, in_block);
    pool_.erase(it);
    return true;
}

bool FeeEstimator::remove_tx(const Uint256& txid, bool in_block) {
    std::lock_guard<std::mutex> g(mu_);
    return remove_locked(txid, in_block);
}

void FeeEstimator::process_block(u32 height, const std::vector<Uint256>& txids) {
    std::lock_guard<std::mutex> g(mu_);
    if (height <= best_seen_) return;   // side chains and reorgs are ignored
    best_seen_ = height;
    for (ConfirmHistory* h : {&med_, &short_, &long_}) {
        h->roll(height);
        h->decay_all();
    }
    unsigned counted = 0;
    for (const Uint256& id : txids) {
        auto it = pool_.find(id);
        if (it == pool_.end()) continue;
        const Tracked t = it->second;
        remove_locked(id, true);
        const int blocks = int(height) - int(t.height);
        if (blocks <= 0) continue;
        med_.record(blocks, t.bucket, t.feerate);
        short_.record(blocks, t.bucket, t.feerate);
        long_.record(blocks, t.bucket, t.feerate);
        ++counted;
    }
    if (first_recorded_ == 0 && counted > 0) first_recorded_ = best_seen_;
}

void FeeEstimator::flush_unconfirmed() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<Uint256> ids;
    ids.reserve(pool_.size());
    for (const auto& kv : pool_) ids.push_back(kv.first);
    for (const Uint256& id : ids) remove_locked(id, false);
}

size_t FeeEstimator::tracked() const {
    std::lock_guard<std::mutex> g(mu_);
    return pool_.size();
}

unsigned FeeEstimator::block_span() const {
    return first_recorded_ == 0 ? 0 : best_seen_ - first_recorded_;
}

unsigned FeeEstimator::historical_span() const {
    if (hist_first_ == 0) return 0;
    if (best_seen_ - hist_best_ > kOldestHistory) return 0;
    return hist_best_ - hist_first_;
}

unsigned FeeEstimator::max_usable_estimate() const {
    return std::min(long_.max_confirms(), std::max(block_span(), historical_span()) / 2);
}

unsigned FeeEstimator::highest_target_tracked(FeeHorizon h) const { return horizon(h).max_confirms(); }

int64_t FeeEstimator::estimate_fee(int target) const {
    if (target <= 1) return 0;
    return estimate_raw_fee(target, kDoubleSuccess, FeeHorizon::Medium, nullptr);
}

int64_t FeeEstimator::estimate_raw_fee(int target, double threshold, FeeHorizon h, FeeEstimation* out) const {
    const ConfirmHistory& s = horizon(h);
    const double sufficient = h == FeeHorizon::Short ? kSufficientTxsShort : kSufficientFeeTxs;
    std::lock_guard<std::mutex> g(mu_);
    if (target <= 0 || unsigned(target) > s.max_confirms() || threshold > 1) return 0;
    const double med = s.median(target, sufficient, threshold, best_seen_, out);
    return med < 0 ? 0 : int64_t(std::llround(med));
}

double FeeEstimator::combined(unsigned target, double success, bool check_shorter, FeeEstimation* out) const {
    double est = -1;
    if (target < 1 || target > long_.max_confirms()) return est;
    if (target <= short_.max_confirms())
        est = short_.median(int(target), kSufficientTxsShort, success, best_seen_, out);
    else if (target <= med_.max_confirms())
        est = med_.median(int(target), kSufficientFeeTxs, success, best_seen_, out);
    else
        est = long_.median(int(target), kSufficientFeeTxs, success, best_seen_, out);
    if (check_shorter) {   // a lower answer from a more recent horizon at its longest target wins
        FeeEstimation tmp;
        if (target > med_.max_confirms()) {
            const double m = med_.median(int(med_.max_confirms()), kSufficientFeeTxs, success, best_seen_, &tmp);
            if (m > 0 && (est == -1 || m < est)) {
                est = m;
                if (out) *out = tmp;
            }
        }
        if (target > short_.max_confirms()) {
            const double m = short_.median(int(short_.max_confirms()), kSufficientTxsShort, success, best_seen_, &tmp);
            if (m > 0 && (est == -1 || m < est)) {
                est = m;
                if (out) *out = tmp;
            }
        }
    }
    return est;
}

double FeeEstimator::conservative(unsigned double_target, FeeEstimation* out) const {
    double est = -1;
    FeeEstimation tmp;
    if (double_target <= short_.max_confirms())
        est = med_.median(int(double_target), kSufficientFeeTxs, kDoubleSuccess, best_seen_, out);
    if (double_target <= med_.max_confirms()) {
        const double l = long_.median(int(double_target), kSufficientFeeTxs, kDoubleSuccess, best_seen_, &tmp);
        if (l > est) {
            est = l;
            if (out) *out = tmp;
        }
    }
    return est;
}

int64_t FeeEstimator::estimate_smart_fee(int target, bool conservative_mode, int* returned_target, FeeReason* reason,
                                         FeeEstimation* out) const {
    std::lock_guard<std::mutex> g(mu_);
    if (returned_target) *returned_target = target;
    if (reason) *reason = FeeReason::None;
    if (target <= 0 || unsigned(target) > long_.max_confirms()) return 0;
    if (target == 1) target = 2;   // a next-block estimate is not possible
    const unsigned usable = max_usable_estimate();
    if (unsigned(target) > usable) target = int(usable);
    if (returned_target) *returned_target = target;
    if (target <= 1) return 0;

    FeeEstimation tmp;
    auto take = [&](double v, double& best, FeeReason why) {
        if (v > best) {
            best = v;
            if (out) *out = tmp;
            if (reason) *reason = why;
        }
    };
    double med = combined(unsigned(target) / 2, kHalfSuccess, true, &tmp);
    if (out) *out = tmp;
    if (reason) *reason = FeeReason::HalfEstimate;
    take(combined(unsigned(target), kSuccess, true, &tmp), med, FeeReason::FullEstimate);
    take(combined(2 * unsigned(target), kDoubleSuccess, !conservative_mode, &tmp), med, FeeReason::DoubleEstimate);
    if (conservative_mode || med == -1)
        take(conservative(2 * unsigned(target), &tmp), med, FeeReason::Conservative);
    return med < 0 ? 0 : int64_t(std::llround(med));
}

Bytes FeeEstimator::serialize() const {
    std::lock_guard<std::mutex> g(mu_);
    Writer w;
    w.i32_(kFileVersion);
    w.i32_(kClientVersion);
    w.u32_(best_seen_);
    if (block_span() > historical_span() / 2) {
        w.u32_(first_recorded_);
        w.u32_(best_seen_);
    } else {
        w.u32_(hist_first_);
        w.u32_(hist_best_);
    }
    put_vec(w, bounds_.data(), bounds_.size());
    med_.write(w);
    short_.write(w);
    long_.write(w);
    return w.buf;
}

bool FeeEstimator::deserialize(const Bytes& b, std::string* err) {
    std::lock_guard<std::mutex> g(mu_);
    try {
        Reader r(b);
        const int required = r.i32_();
        const int wrote = r.i32_();
        if (required > kClientVersion) throw std::runtime_error("up-version fee estimate file");
        const u32 best = r.u32_();
        if (wrote < kFileVersion) throw std::runtime_error("pre-0.15 fee estimate file (discarded, as the reference)");
        const u32 hfirst = r.u32_(), hbest = r.u32_();
        if (hfirst > hbest || hbest > best)
            throw std::runtime_error("Corrupt estimates file. Historical block range for estimates is invalid");
        std::vector<double> bounds = get_vec(r);
        if (bounds.size() <= 1 || bounds.size() > 1000)
            throw std::runtime_error("Corrupt estimates file. Must have between 2 and 1000 feerate buckets");
        // parse into temporaries first so a corrupt file leaves the live state untouched
        std::vector<double> keep = bounds;
        ConfirmHistory m(&bounds_, kMedPeriods, kMedDecay, kMedScale), s(&bounds_, kShortPeriods, kShortDecay, kShortScale),
            l(&bounds_, kLongPeriods, kLongDecay, kLongScale);
        m.read(r, bounds.size());
        s.read(r, bounds.size());
        l.read(r, bounds.size());
        bounds_ = std::move(keep);
        med_ = m;
        short_ = s;
        long_ = l;
        pool_.clear();
        best_seen_ = best;
        hist_first_ = hfirst;
        hist_best_ = hbest;
        first_recorded_ = 0;
        return true;
    } catch (const std::exception& e) {
        if (err) *err = e.what();
        return false;
    }
}

}  // namespace nodexa
