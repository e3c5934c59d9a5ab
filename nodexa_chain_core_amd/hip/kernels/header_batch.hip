// Device-resident batch header verification: the glue kernels of the pipeline in models/verify.py
// (verify_batch_resident; BASELINE config 5). Reference behaviour: CheckBlockHeader
// (src/validation.cpp:11638-11665: full KawPow and mix_hash equality) applied to every header of a
// `headers` message, which the reference does serially under cs_main (:12017-12035).
//
// The batch is uploaded once as 128-byte rows (csrc/chain/headerbatch.hpp); then, on one stream
// with no host round trip:
//   kawpow_mixonly_batch (sha256d.hip)  rows -> header hash | mix-only final | boundary | claimed mix
//   hb_jobs                             -> KawpowVerifyJob + program index per header
//   kawpow_verify_dag (per epoch range) -> computed mix | final per header (the resident DAG)
//   hb_verdict                          -> one code per KawPow header
//   eq_verify + sha256d_batch + hb_eq_scatter for Equihash-extension headers (side stream)
//   dgw_batch                           -> the DarkGravityWave nBits of every header (side stream)
// hb_jobs writes the KawPow block hashes, so hashes + nBits are complete once the side stream and
// hb_jobs are done: an early copy of them lets the host prepare the index insert while the full
// hashes run, and one final device-to-host copy brings back codes, hashes and nBits together.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_params.h"

#define HB_ROW 128

__device__ __forceinline__ uint32_t hb_le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// One thread per header: the verify job of a KawPow row (header hash from the mix-only pass,
// nNonce64 / nHeight from the row) and its program's index in its epoch's resident program table
// (period - epoch * periods_per_epoch). Other kinds get a harmless job (program 0).
extern "C" __global__ __launch_bounds__(256) void hb_jobs(HeaderBatchParams p) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= p.count) return;
    const uint32_t i = p.first + t;
    const uint8_t* row = p.rows + (size_t)i * HB_ROW;
    const uint8_t* mo = p.mixonly + (size_t)i * 128;
    KawpowVerifyJob j;
#pragma unroll
    for (int k = 0; k < 8; ++k) j.header[k] = hb_le32(mo + 4 * k);
    const uint32_t height = hb_le32(row + 76);
    j.nonce = (uint64_t)hb_le32(row + 80) | ((uint64_t)hb_le32(row + 84) << 32);
    j.block_number = height;
    j.pad = 0;
    uint32_t prog = 0;
    if (p.kinds[i] == 0) {
        const uint32_t period = height / 3u, epoch = height / p.epoch_length;
        prog = period - epoch * (p.epoch_length / 3u);
    }
    p.jobs[i] = j;
    p.job_program[i] = prog;
    // a KawPow row's block hash (GetHash: the mix-only final, byte-reversed into uint256 storage
    // order) is known here already: written now, the early copy of hashes + nBits lets the host
    // prepare the index insert while the full hashes are still running
    if (p.kinds[i] == 0) {
        uint8_t* out_hash = p.out + (size_t)p.n + (size_t)i * 32;
#pragma unroll
        for (int k = 0; k < 32; ++k) out_hash[k] = mo[32 + 31 - k];
    }
}

// One thread per header: the verdict of a KawPow row from the mix-only pass and the full hash
// (kawpow::verify: the claimed mix must meet the boundary, then the recomputed mix must equal it),
// and the block hash (GetHash: the mix-only final, byte-reversed into uint256 storage order).
// Codes: 0 valid, 1 invalid-mix-hash, 2 high-hash, 255 another kind (filled in later or by the host).
extern "C" __global__ __launch_bounds__(256) void hb_verdict(HeaderBatchParams p) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= p.count) return;
    const uint32_t i = p.first + t;
    const uint8_t* mo = p.mixonly + (size_t)i * 128;
    if (p.kinds[i] != 0) {
        // Equihash rows get their code from hb_eq_scatter (on the side stream, possibly already
        // done); pre-KawPow rows are decided by the host
        if (p.kinds[i] != 2) p.out[i] = 255;
        return;
    }
    // CheckBlockHeader's order (src/validation.cpp:11638-11665): below the last checkpoint only the
    // cheap mix-only hash (GetHash) must meet nBits; above it the full hash (GetHashFull) must meet
    // nBits ("high-hash") and then its mix must equal the claimed one ("invalid-mix-hash")
    const uint32_t height = hb_le32(p.rows + (size_t)i * HB_ROW + 76);
    const bool below_cp = p.last_checkpoint >= 0 && (int64_t)height <= (int64_t)p.last_checkpoint;
    const uint32_t* full = p.full + (size_t)i * 16;  // computed mix words 0..7, final 8..15
    int cmp = 0;  // final <= boundary, both big-endian 256-bit (ethash is_less_or_equal)
    for (int k = 0; k < 32 && cmp == 0; ++k) {
        const uint8_t a = below_cp ? mo[32 + k] : (uint8_t)(full[8 + k / 4] >> (8 * (k & 3)));
        const uint8_t b = mo[64 + k];
        cmp = a < b ? -1 : (a > b ? 1 : 0);
    }
    // CheckProofOfWork also refuses a target above powLimit (the boundary is big-endian here)
    int lim = 0;
    for (int k = 0; k < 32 && lim == 0; ++k) {
        const uint8_t a = mo[64 + k], b = p.pow_limit[31 - k];
        lim = a < b ? -1 : (a > b ? 1 : 0);
    }
    uint8_t code = (cmp <= 0 && lim <= 0) ? 0 : 2;
    if (code == 0 && !below_cp) {
        bool same = true;
#pragma unroll
        for (int k = 0; k < 8; ++k) same &= full[k] == hb_le32(mo + 96 + 4 * k);
        code = same ? 0 : 1;
    }
    p.out[i] = code;  // (the block hash was written by hb_jobs)
}

// Equihash-extension headers: the eq_verify verdict (0 = valid solution) and the SHA256d block
// hash meeting nBits decide the code (0 / 3 invalid-solution / 2 high-hash); both land at the
// header's batch position.
extern "C" __global__ __launch_bounds__(256) void hb_eq_scatter(HeaderBatchParams p) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= p.eq_n) return;
    const uint32_t i = p.eq_index[k];
    const uint8_t* h = p.eq_hash + (size_t)k * 32;  // SHA256d digest = uint256 storage order
    uint8_t* out_hash = p.out + (size_t)p.n + (size_t)i * 32;
    // CheckProofOfWork: hash (little-endian 256-bit) <= SetCompact(nBits)
    const uint32_t bits = hb_le32(p.rows + (size_t)i * HB_ROW + 72);
    const uint32_t ex = bits >> 24;
    uint32_t mant = bits & 0x007fffffu;
    const bool neg = mant != 0 && (bits & 0x00800000u) != 0;
    const bool ovf = mant != 0 && (ex > 34 || (mant > 0xff && ex > 33) || (mant > 0xffff && ex > 32));
    uint8_t t[32];  // little-endian target bytes
#pragma unroll
    for (int q = 0; q < 32; ++q) t[q] = 0;
    if (ex <= 3) {
        mant >>= 8 * (3 - ex);
        t[0] = uint8_t(mant); t[1] = uint8_t(mant >> 8); t[2] = uint8_t(mant >> 16);
    } else {
        for (uint32_t q = 0; q < 3; ++q)
            if (ex - 3 + q < 32) t[ex - 3 + q] = uint8_t(mant >> (8 * q));
    }
    bool le = true;  // compare from the most significant byte
    for (int q = 31; q >= 0; --q) {
        if (h[q] != t[q]) {
            le = h[q] < t[q];
            break;
        }
    }
    bool above = false;  // target > powLimit
    for (int q = 31; q >= 0; --q) {
        if (t[q] != p.pow_limit[q]) {
            above = t[q] > p.pow_limit[q];
            break;
        }
    }
    const bool zero_target = neg || ovf || (mant == 0);
    uint8_t code = p.eq_verdict[k] != 0 ? 3 : ((!zero_target && !above && le) ? 0 : 2);
    p.out[i] = code;
#pragma unroll
    for (int q = 0; q < 32; ++q) out_hash[q] = h[q];
}
