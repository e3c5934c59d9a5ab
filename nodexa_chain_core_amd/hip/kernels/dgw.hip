// Batch DarkGravityWave v3 for gfx950: one thread per header of a linear header
// batch computes the nBits that header must carry, from the 180 (nTime, nBits) pairs before it.
//
// Reference: DarkGravityWave (src/pow.cpp:18-102), serial per header under cs_main. The host
// model is csrc/chain/pow_rules.cpp dgw_average; this kernel is its bit-exact twin, checked
// against it over a 10k-header fixture in tests/test_gpu_verify.py:
//   * the running "average" avg = (avg * count + target) / (count + 1) over the 180 blocks,
//     newest first, on 32-bit limbs with the reference's mod-2^256 wrap-around, the division by
//     count + 1 <= 181 exact through a 64-bit reciprocal (every partial dividend is < d * 2^32);
//   * the KawPow / Equihash switch bootstraps (any non-KawPow block in the window -> the KawPow
//     limit, likewise for the Equihash extension);
//   * the 1/3x..3x clamp of the actual timespan, bn *= actual, bn /= 180 * spacing, the pow limit
//     cap and GetCompact.
// Each thread reads 2 x 180 words that neighbouring threads read too (the series is shared), so
// the loads come from L2 / L1; the cost is the ~2 x 8 dependent limb operations per step.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_params.h"

#ifndef NX_DEV
#define NX_DEV __device__ __forceinline__
#endif

namespace {

constexpr int kPast = 180;

NX_DEV void set_compact(uint32_t r[8], uint32_t compact) {
    const int size = int(compact >> 24);
    uint32_t word = compact & 0x007fffffu;
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = 0;
    if (size <= 3) {
        r[0] = word >> (8 * (3 - size));
        return;
    }
    const unsigned shift = unsigned(8 * (size - 3));
    const unsigned k = shift / 32, b = shift % 32;
    if (k < 8) r[k] = word << b;
    if (b != 0 && k + 1 < 8) r[k + 1] = word >> (32 - b);
}

NX_DEV int bit_length(const uint32_t a[8]) {
    for (int i = 7; i >= 0; --i)
        if (a[i]) return 32 * i + (32 - __clz(a[i]));
    return 0;
}

NX_DEV uint32_t get_compact(const uint32_t a[8]) {
    int size = (bit_length(a) + 7) / 8;
    uint32_t compact;
    if (size <= 3) {
        const uint64_t low = (uint64_t(a[1]) << 32) | a[0];
        compact = uint32_t(low << (8 * (3 - size)));
    } else {
        const unsigned shift = unsigned(8 * (size - 3));
        const unsigned k = shift / 32, b = shift % 32;
        // the low 32 bits of a >> shift
        uint32_t lo = k < 8 ? a[k] >> b : 0;
        if (b != 0 && k + 1 < 8) lo |= a[k + 1] << (32 - b);
        compact = lo;
    }
    if (compact & 0x00800000u) {
        compact >>= 8;
        size++;
    }
    return compact | (uint32_t(size) << 24);
}

// avg = (avg * count + t) / (count + 1), mod 2^256 before the division (operator*(uint32) and +)
NX_DEV void dgw_step(uint32_t a[8], uint32_t count, const uint32_t t[8], const uint64_t* recip) {
    uint64_t carry = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        carry += uint64_t(a[i]) * count + t[i];
        a[i] = uint32_t(carry);
        carry >>= 32;
    }
    const uint64_t d = count + 1, m = recip[d];  // ceil(2^64 / d)
    uint64_t rem = 0;
#pragma unroll
    for (int i = 7; i >= 0; --i) {
        const uint64_t cur = (rem << 32) | a[i];
        const uint64_t q = __umul64hi(cur, m);
        rem = cur - q * d;
        a[i] = uint32_t(q);
    }
}

NX_DEV bool greater(const uint32_t a[8], const uint32_t b[8]) {
    for (int i = 7; i >= 0; --i)
        if (a[i] != b[i]) return a[i] > b[i];
    return false;
}

}  // namespace

extern "C" __global__ __launch_bounds__(256) void dgw_batch(DgwParams p) {
    __shared__ uint64_t recip[kPast + 2];  // ceil(2^64 / d), d = 2..181, one division per thread
    for (uint32_t d = threadIdx.x; d < kPast + 2; d += blockDim.x) recip[d] = d >= 2 ? ~0ull / d + 1 : 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.n) return;
    const int last_height = p.base_height + int(i);  // height of header i's parent
    if (last_height + 1 < p.dgw_activation_block) {
        p.out[i] = 0;  // BTC retarget era: the host's serial path
        return;
    }
    if (last_height < kPast) {
        p.out[i] = p.pow_limit_compact;
        return;
    }
    const int64_t j = int64_t(p.a) - 1 + int64_t(i);  // series index of header i's parent
    if (j < kPast - 1) {  // the series does not reach back 180 blocks: let the host decide
        p.out[i] = 0;
        return;
    }
    uint32_t avg[8], t[8];
    int kawpow_blocks = 0, equihash_blocks = 0;
    for (uint32_t count = 1; count <= uint32_t(kPast); ++count) {
        const int64_t k = j - int64_t(count - 1);
        set_compact(t, p.bits[k]);
        if (count == 1) {
#pragma unroll
            for (int q = 0; q < 8; ++q) avg[q] = t[q];
        } else {
            dgw_step(avg, count, t, recip);
        }
        const uint32_t tk = p.times[k];
        kawpow_blocks += tk >= p.kawpow_time;
        equihash_blocks += tk >= p.equihash_time;
    }
    const uint32_t next_time = p.times[j + 1];
    if (next_time >= p.equihash_time && equihash_blocks != kPast) {
        p.out[i] = p.equihash_limit_compact;
        return;
    }
    if (next_time >= p.kawpow_time && kawpow_blocks != kPast) {
        p.out[i] = p.kawpow_limit_compact;
        return;
    }
    int64_t actual = int64_t(p.times[j]) - int64_t(p.times[j - (kPast - 1)]);
    const int64_t span = p.target_timespan;
    if (actual < span / 3) actual = span / 3;
    if (actual > span * 3) actual = span * 3;
    // bn *= uint32(actual) (mod 2^256), then bn /= span (exact long division, 32-bit limbs)
    uint64_t carry = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        carry += uint64_t(avg[q]) * uint32_t(actual);
        avg[q] = uint32_t(carry);
        carry >>= 32;
    }
    uint64_t rem = 0;
    const uint64_t d = uint64_t(span);
#pragma unroll
    for (int q = 7; q >= 0; --q) {
        const uint64_t cur = (rem << 32) | avg[q];
        avg[q] = uint32_t(cur / d);
        rem = cur % d;
    }
    if (greater(avg, p.pow_limit)) {
        p.out[i] = p.pow_limit_compact;
        return;
    }
    p.out[i] = get_compact(avg);
}
