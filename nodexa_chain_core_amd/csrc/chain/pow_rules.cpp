#include "pow_rules.hpp"

#include <algorithm>
#include <array>
#include <cmath>
#include <stdexcept>

namespace nodexa {

int64_t HeaderIndex::median_time_past() const {
    int64_t times[11];
    int n = 0;
    for (const HeaderIndex* p = this; p && n < 11; p = p->prev) times[n++] = p->time;
    std::sort(times, times + n);
    return times[n / 2];
}

const HeaderIndex* HeaderIndex::ancestor(int h) const {
    if (h > height || h < 0) return nullptr;
    const HeaderIndex* p = this;
    while (p && p->height > h) p = (p->skip && p->skip->height >= h) ? p->skip : p->prev;
    return p;
}

namespace {

// One step of DGW's running "average", avg = (avg * count + target) / (count + 1), on the
// 32-bit limbs with the reference's wrap-around (operator*(uint32_t) and operator+ are
// mod 2^256) and an exact limb-wise division by the small divisor through a 64-bit
// reciprocal: every partial dividend is < d * 2^32 and d <= 181, so
// floor(x * ceil(2^64 / d) / 2^64) == floor(x / d) (the error term stays < d / 2^32,
// below the 1/d gap to the next integer). ~5x faster than the generic long division.
constexpr u32 kDgwMaxDivisor = 181;

const u64* dgw_reciprocals() {
    static const auto tbl = [] {
        std::array<u64, kDgwMaxDivisor + 1> t{};
        for (u32 d = 2; d <= kDgwMaxDivisor; ++d) t[d] = ~u64(0) / d + 1;
        return t;
    }();
    return tbl.data();
}

inline void dgw_step(u32 a[8], u32 count, const u32 t[8], const u64* recip) {
    u64 carry = 0;
    for (int i = 0; i < 8; ++i) {
        carry += u64(a[i]) * count + t[i];
        a[i] = u32(carry);
        carry >>= 32;
    }
    const u64 d = count + 1, m = recip[d];
    u64 rem = 0;
    for (int i = 7; i >= 0; --i) {
        const u64 cur = (rem << 32) | a[i];
        const u64 q = u64((unsigned __int128)cur * m >> 64);
        rem = cur - q * d;
        a[i] = u32(q);
    }
}

}  // namespace

u32 dgw_average(const u32* times, const u32* bits, int64_t j, u32 next_time, const ChainParams& params) {
    const ConsensusParams& c = params.consensus;
    constexpr int64_t past_blocks = kDgwPastBlocks;
    static_assert(past_blocks < kDgwMaxDivisor, "reciprocal table too small");
    if (j < past_blocks - 1) throw std::logic_error("DGW window shorter than 180 blocks");
    const u64* recip = dgw_reciprocals();
    ArithU256 avg;
    int kawpow_blocks = 0, equihash_blocks = 0;
    for (u32 count = 1; count <= u32(past_blocks); ++count) {
        const int64_t k = j - int64_t(count - 1);
        ArithU256 target;
        target.set_compact(bits[k]);
        if (count == 1) avg = target;
        else dgw_step(avg.pn, count, target.pn, recip);  // "not really an average" (src/pow.cpp:57)
        if (times[k] >= params.kawpow_activation_time) ++kawpow_blocks;
        if (times[k] >= params.equihash_activation_time) ++equihash_blocks;
    }
    // Equihash extension (new): same bootstrap as the KawPow switch below
    if (next_time >= params.equihash_activation_time && equihash_blocks != past_blocks)
        return ArithU256::from_uint256(c.equihash_limit.is_null() ? c.pow_limit : c.equihash_limit).get_compact();
    if (next_time >= params.kawpow_activation_time && kawpow_blocks != past_blocks)
        return ArithU256::from_uint256(c.kawpow_limit).get_compact();

    const ArithU256 pow_limit = ArithU256::from_uint256(c.pow_limit);
    ArithU256 bn = avg;
    int64_t actual = int64_t(times[j]) - int64_t(times[j - (past_blocks - 1)]);
    const int64_t target_timespan = past_blocks * c.pow_target_spacing;
    if (actual < target_timespan / 3) actual = target_timespan / 3;
    if (actual > target_timespan * 3) actual = target_timespan * 3;
    bn *= u32(actual);                        // operator*=(uint32_t) in the reference
    bn /= ArithU256(u64(target_timespan));    // operator/=(base_uint(uint64))
    if (bn > pow_limit) bn = pow_limit;
    return bn.get_compact();
}

u32 dark_gravity_wave(const HeaderIndex* last, const BlockHeader& next, const ChainParams& params) {
    const ConsensusParams& c = params.consensus;
    const u32 pow_limit_compact = ArithU256::from_uint256(c.pow_limit).get_compact();
    if (!last || last->height < kDgwPastBlocks) return pow_limit_compact;

    if (c.pow_allow_min_difficulty_blocks && c.pow_no_retargeting) {
        if (int64_t(next.time) > int64_t(last->time) + c.pow_target_spacing * 2) return pow_limit_compact;
        const HeaderIndex* p = last;
        while (p->prev && p->height % c.difficulty_adjustment_interval() != 0 && p->bits == pow_limit_compact)
            p = p->prev;
        return p->bits;
    }
    u32 times[kDgwPastBlocks], bits[kDgwPastBlocks];
    const HeaderIndex* p = last;
    for (int k = kDgwPastBlocks - 1; k >= 0; --k) {
        times[k] = p->time;
        bits[k] = p->bits;
        if (k) {
            if (!p->prev) throw std::logic_error("DGW walked past genesis");
            p = p->prev;
        }
    }
    return dgw_average(times, bits, kDgwPastBlocks - 1, next.time, params);
}

u32 calculate_next_work_required(const HeaderIndex* last, int64_t first_block_time, const ChainParams& params) {
    const ConsensusParams& c = params.consensus;
    if (c.pow_no_retargeting) return last->bits;
    int64_t actual = int64_t(last->time) - first_block_time;
    if (actual < c.pow_target_timespan / 4) actual = c.pow_target_timespan / 4;
    if (actual > c.pow_target_timespan * 4) actual = c.pow_target_timespan * 4;
    const ArithU256 pow_limit = ArithU256::from_uint256(c.pow_limit);
    ArithU256 bn;
    bn.set_compact(last->bits);
    bn *= u32(actual);
    bn /= ArithU256(u64(c.pow_target_timespan));
    if (bn > pow_limit) bn = pow_limit;
    return bn.get_compact();
}

u32 next_work_required_btc(const HeaderIndex* last, const BlockHeader& next, const ChainParams& params) {
    const ConsensusParams& c = params.consensus;
    const u32 pow_limit_compact = ArithU256::from_uint256(c.pow_limit).get_compact();
    const int64_t interval = c.difficulty_adjustment_interval();
    if ((last->height + 1) % interval != 0) {
        if (c.pow_allow_min_difficulty_blocks) {
            if (int64_t(next.time) > int64_t(last->time) + c.pow_target_spacing * 2) return pow_limit_compact;
            const HeaderIndex* p = last;
            while (p->prev && p->height % interval != 0 && p->bits == pow_limit_compact) p = p->prev;
            return p->bits;
        }
        return last->bits;
    }
    const int first_height = last->height - int(interval - 1);
    const HeaderIndex* first = last->ancestor(first_height);
    if (!first) throw std::logic_error("BTC retarget: missing ancestor");
    return calculate_next_work_required(last, first->time, params);
}

u32 next_work_required(const HeaderIndex* last, const BlockHeader& next, const ChainParams& params) {
    // IsDGWActive(nHeight) = nHeight >= nDGWActivationBlock
    if (last->height + 1 >= params.dgw_activation_block) return dark_gravity_wave(last, next, params);
    return next_work_required_btc(last, next, params);
}

bool check_proof_of_work(const Uint256& hash, u32 bits, const ChainParams& params) {
    bool negative = false, overflow = false;
    ArithU256 target;
    target.set_compact(bits, &negative, &overflow);
    if (negative || target.is_zero() || overflow || target > ArithU256::from_uint256(params.consensus.pow_limit))
        return false;
    return !(ArithU256::from_uint256(hash) > target);
}

ArithU256 block_proof(u32 bits) {
    bool negative = false, overflow = false;
    ArithU256 target;
    target.set_compact(bits, &negative, &overflow);
    if (negative || overflow || target.is_zero()) return ArithU256();
    // 2**256 / (target+1) == ~target / (target+1) + 1
    const ArithU256 num = ~target, d = target + ArithU256(1);
    const unsigned L = d.bits();
    if (L < 193) return (num / d) + ArithU256(1);
    // Every real target is >= 2^192, so the quotient fits in 64 bits: estimate it from the top
    // 64 bits of d (rounded up, so the estimate never exceeds the quotient and d * q cannot
    // wrap) and the matching top bits of the numerator (< 2^128), then correct upward by the
    // remainder. The estimate is at most a few units low, so this is exact in a few steps --
    // much cheaper than the bit-serial long division (block proofs are computed for every
    // header of every batch).
    const unsigned s = L - 64;
    const ArithU256 nh = num >> s;
    const unsigned __int128 top = (static_cast<unsigned __int128>((nh >> 64).low64()) << 64) | nh.low64();
    const unsigned __int128 q128 = top / (static_cast<unsigned __int128>((d >> s).low64()) + 1);
    u64 q = u64(q128);
    ArithU256 rem = num - (d * u32(q) + ((d * u32(q >> 32)) << 32));
    while (rem >= d) {
        rem -= d;
        ++q;
    }
    return ArithU256(q) + ArithU256(1);
}

Amount block_subsidy(int height) {
    // Linux/glibc branch of the reference (the Windows branch patches libm
    // differences with a lookup table of these same values).
    const Amount s = Amount(54193019856 * std::pow(1 - 0.00000041686938347033551682078457954749861613663597381673753261566162109375,
                                                   height));
    return s;
}

double difficulty_from_bits(u32 bits) {
    int shift = (bits >> 24) & 0xff;
    double diff = double(0x0000ffff) / double(bits & 0x00ffffff);
    while (shift < 29) { diff *= 256.0; ++shift; }
    while (shift > 29) { diff /= 256.0; --shift; }
    return diff;
}

}  // namespace nodexa
