// Ethash dataset (DAG) generation on gfx950.
//
// Each 512-bit item (src/crypto/ethash/lib/ethash/ethash.cpp:180-207):
//   mix = keccak512(light[i % n] with word0 ^= i)
//   512 x { parent = fnv1(i ^ j, mix[j % 16]) % n ; mix = fnv1(mix, light[parent]) }
//   item = keccak512(mix)
// The light cache (16 MiB at epoch 0 .. 64 MiB at epoch 384) stays resident in the 256 MiB
// Infinity Cache, and the build is bound by its rate for random 64-byte reads.
//
// CDNA4 mapping: one item per aligned lane quad. Lane s of the quad owns mix words 4s..4s+3 and
// reads its 16 bytes of every parent, so a wave-wide parent load is one 16-byte load per lane
// touching 16 lines, each read whole by its quad (a thread-per-item layout needs four 16-byte
// loads per lane touching 64 lines each for the same bytes). The parent index word mix[j % 16]
// lives in quad lane (j % 16) / 4 and reaches the other three by a DPP quad_perm broadcast (j % 16
// is a literal after unrolling by 16). Each lane runs the two keccak512s itself: VALU the build
// has to spare. tools/dag_build_probe.hip (profiles/r6m_rehearsal): 3.80 TB/s of parent reads at
// epoch 384 against 3.46 for thread-per-item, i.e. the measured ceiling for independent random
// 64-byte reads of a 64 MiB buffer (3.68 TB/s); 4 GiB in 0.578 s instead of 0.636.
#include "kernel_params.h"
#include "keccak_device.hpp"

NX_DEV uint32_t fnv1(uint32_t u, uint32_t v) { return (u * 0x01000193u) ^ v; }

NX_DEV uint32_t dag_mod(uint32_t x, const FastMod32& f) {
    const uint32_t r = x - __umulhi(x, f.mb) * f.d;  // Barrett estimate, one correction (kernel_params.h)
    return min(r, r - f.d);
}

// lane C of each aligned quad, to the whole quad
template <int C>
NX_DEV uint32_t dag_quad_bcast(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, C * 0x55, 0xf, 0xf, false);
}

// 64 items per 256-thread workgroup; the host launches ceil(num_items / 64) workgroups
extern "C" __global__ __launch_bounds__(256) void ethash_dag_build(EthashDagParams p, FastMod32 lmod) {
    const uint64_t local = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
    if (local >= p.num_items) return;  // whole quads: the quad's lanes share `local`
    const uint32_t s = threadIdx.x & 3;
    const uint64_t index = p.first_item + local;
    const uint4* __restrict__ light = (const uint4*)p.light;
    const uint32_t seed = (uint32_t)index;  // index < 2^32 for every supported epoch

    uint32_t m[4];
    {
        const uint32_t li = dag_mod(seed, lmod);
        uint64_t in[8], out[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v = light[(size_t)li * 4 + k];
            in[2 * k] = ((uint64_t)v.y << 32) | v.x;
            in[2 * k + 1] = ((uint64_t)v.w << 32) | v.z;
        }
        in[0] ^= seed;
        keccak512_64(in, out);
        const uint64_t lo = (s & 2) ? ((s & 1) ? out[6] : out[4]) : ((s & 1) ? out[2] : out[0]);
        const uint64_t hi = (s & 2) ? ((s & 1) ? out[7] : out[5]) : ((s & 1) ? out[3] : out[1]);
        m[0] = (uint32_t)lo;
        m[1] = (uint32_t)(lo >> 32);
        m[2] = (uint32_t)hi;
        m[3] = (uint32_t)(hi >> 32);
    }

#pragma unroll 1
    for (uint32_t j = 0; j < 512; j += 16) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t own = m[k & 3];
            uint32_t mk;
            switch (k >> 2) {
                case 0: mk = dag_quad_bcast<0>(own); break;
                case 1: mk = dag_quad_bcast<1>(own); break;
                case 2: mk = dag_quad_bcast<2>(own); break;
                default: mk = dag_quad_bcast<3>(own); break;
            }
            const uint32_t parent = dag_mod(fnv1(seed ^ (j + (uint32_t)k), mk), lmod);
            const uint4 v = light[(size_t)parent * 4 + s];
            m[0] = fnv1(m[0], v.x);
            m[1] = fnv1(m[1], v.y);
            m[2] = fnv1(m[2], v.z);
            m[3] = fnv1(m[3], v.w);
        }
    }

    // final keccak512 over the whole 16-word mix, gathered from the quad
    uint32_t all[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        all[k] = dag_quad_bcast<0>(m[k]);
        all[4 + k] = dag_quad_bcast<1>(m[k]);
        all[8 + k] = dag_quad_bcast<2>(m[k]);
        all[12 + k] = dag_quad_bcast<3>(m[k]);
    }
    uint64_t in[8], out[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) in[k] = ((uint64_t)all[2 * k + 1] << 32) | all[2 * k];
    keccak512_64(in, out);
    const uint64_t lo = (s & 2) ? ((s & 1) ? out[6] : out[4]) : ((s & 1) ? out[2] : out[0]);
    const uint64_t hi = (s & 2) ? ((s & 1) ? out[7] : out[5]) : ((s & 1) ? out[3] : out[1]);
    // absolute item index: shards build in place
    ((uint4*)p.dag)[index * 4 + s] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}
