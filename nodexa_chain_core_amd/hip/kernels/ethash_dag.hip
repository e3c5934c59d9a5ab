// Ethash dataset (DAG) generation on gfx950.
//
// One 512-bit item per thread (src/crypto/ethash/lib/ethash/ethash.cpp:180-207):
//   mix = keccak512(light[i % n] with word0 ^= i)
//   512 x { parent = fnv1(i ^ j, mix[j % 16]) % n ; mix = fnv1(mix, light[parent]) }
//   item = keccak512(mix)
// The light cache (16 MiB at epoch 0 .. 64 MiB at epoch 384) stays resident in
// the 256 MiB Infinity Cache, so the 512 dependent 64-byte parent gathers per
// item are served on-die; the loop is unrolled by 16 so `mix[j % 16]` is a
// register, never a runtime-indexed (scratch) array. `% n` uses the FastMod32
// round-up reciprocal instead of a 32-bit divide.
#include "kernel_params.h"
#include "keccak_device.hpp"

NX_DEV uint32_t fastmod(uint32_t x, const FastMod32& f) {
    const uint32_t t = __umulhi(x, f.m);
    const uint32_t q = (t + ((x - t) >> 1)) >> (f.s - 1);
    return x - q * f.d;
}

NX_DEV uint32_t fnv1(uint32_t u, uint32_t v) { return (u * 0x01000193u) ^ v; }

extern "C" __global__ __launch_bounds__(256) void ethash_dag_build(EthashDagParams p, FastMod32 lmod) {
    const uint64_t local = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (local >= p.num_items) return;
    const uint64_t index = p.first_item + local;
    const uint4* __restrict__ light = (const uint4*)p.light;
    const uint32_t seed = (uint32_t)index;

    uint32_t mix[16];
    {
        const uint32_t li = fastmod(seed, lmod);  // index < 2^32 for every supported epoch
        uint64_t in[8], out[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v = light[(size_t)li * 4 + k];
            in[2 * k] = ((uint64_t)v.y << 32) | v.x;
            in[2 * k + 1] = ((uint64_t)v.w << 32) | v.z;
        }
        in[0] ^= seed;
        keccak512_64(in, out);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            mix[2 * k] = (uint32_t)out[k];
            mix[2 * k + 1] = (uint32_t)(out[k] >> 32);
        }
    }

#pragma unroll 1
    for (uint32_t j = 0; j < 512; j += 16) {
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t parent = fastmod(fnv1(seed ^ (j + k), mix[k]), lmod);
            const uint4* src = light + (size_t)parent * 4;
            const uint4 a = src[0], b = src[1], c = src[2], d = src[3];
            mix[0] = fnv1(mix[0], a.x); mix[1] = fnv1(mix[1], a.y);
            mix[2] = fnv1(mix[2], a.z); mix[3] = fnv1(mix[3], a.w);
            mix[4] = fnv1(mix[4], b.x); mix[5] = fnv1(mix[5], b.y);
            mix[6] = fnv1(mix[6], b.z); mix[7] = fnv1(mix[7], b.w);
            mix[8] = fnv1(mix[8], c.x); mix[9] = fnv1(mix[9], c.y);
            mix[10] = fnv1(mix[10], c.z); mix[11] = fnv1(mix[11], c.w);
            mix[12] = fnv1(mix[12], d.x); mix[13] = fnv1(mix[13], d.y);
            mix[14] = fnv1(mix[14], d.z); mix[15] = fnv1(mix[15], d.w);
        }
    }

    uint64_t in[8], out[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) in[k] = ((uint64_t)mix[2 * k + 1] << 32) | mix[2 * k];
    keccak512_64(in, out);
    uint4* dst = (uint4*)p.dag + (size_t)index * 4;  // absolute item index: shards build in place
#pragma unroll
    for (int k = 0; k < 4; ++k)
        dst[k] = make_uint4((uint32_t)out[2 * k], (uint32_t)(out[2 * k] >> 32), (uint32_t)out[2 * k + 1],
                            (uint32_t)(out[2 * k + 1] >> 32));
}
