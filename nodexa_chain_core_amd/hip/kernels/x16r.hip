// X16R / X16RV2 on gfx950 (the legacy-header PoW, src/hash.h:335-605).
//
// The chain applies 16 primitives in an order taken from hashPrevBlock, so consecutive headers of a
// batch run different algorithms at every step. Instead of one lane walking its own chain (a wave's
// 64 lanes would diverge across up to 17 code paths at every step), the batch advances one step at
// a time: the host groups the headers of step s by slot, and x16r_step runs workgroup (x, slot) over
// that slot's group, so every wave executes one primitive with no divergence. The chain value lives
// in an n x 64-byte device buffer between the 16 launches (one stream, no host round trip); the
// final hash is its first 32 bytes. The primitives are hip/kernels/x16r_device.hpp (the host's
// constructions, tables generated from them).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_params.h"

#define X16R_FN __device__ inline
#include "x16r_device.hpp"

#define X16R_BLOCK 64

extern "C" __global__ __launch_bounds__(X16R_BLOCK) void x16r_step(X16rStepParams p) {
    const int slot = (int)blockIdx.y;
    const int32_t lo = p.offsets[slot], hi = p.offsets[slot + 1];
    const int32_t k = lo + (int32_t)(blockIdx.x * X16R_BLOCK + threadIdx.x);
    if (k >= hi) return;
    const uint32_t i = (uint32_t)p.order[k];
    if (i >= p.n) return;
    uint8_t in[80];
    int len;
    if (p.step == 0) {
        const uint4* src = (const uint4*)(p.headers + (size_t)i * 80);
        for (int w = 0; w < 5; ++w) {
            const uint4 v = src[w];
            x16rd::st32(in + 16 * w, v.x);
            x16rd::st32(in + 16 * w + 4, v.y);
            x16rd::st32(in + 16 * w + 8, v.z);
            x16rd::st32(in + 16 * w + 12, v.w);
        }
        len = 80;
    } else {
        const uint4* src = (const uint4*)(p.state + (size_t)i * 64);
        for (int w = 0; w < 4; ++w) {
            const uint4 v = src[w];
            x16rd::st32(in + 16 * w, v.x);
            x16rd::st32(in + 16 * w + 4, v.y);
            x16rd::st32(in + 16 * w + 8, v.z);
            x16rd::st32(in + 16 * w + 12, v.w);
        }
        len = 64;
    }
    uint8_t out[64];
    x16rd::step(slot, p.v2[i] != 0, in, len, out);
    uint4* dst = (uint4*)(p.state + (size_t)i * 64);
    for (int w = 0; w < 4; ++w)
        dst[w] = make_uint4(x16rd::ld32(out + 16 * w), x16rd::ld32(out + 16 * w + 4), x16rd::ld32(out + 16 * w + 8),
                            x16rd::ld32(out + 16 * w + 12));
}
