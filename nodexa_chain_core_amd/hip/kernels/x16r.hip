// X16R / X16RV2 on gfx950 (the legacy-header PoW, src/hash.h:335-605).
//
// The chain applies 16 primitives in an order taken from hashPrevBlock, so consecutive headers of a
// batch run different algorithms at every step. Instead of one lane walking its own chain (a wave's
// 64 lanes would diverge across up to 17 code paths at every step), the batch advances one step at
// a time: the host groups the headers of step s by slot, and that slot's kernel runs over the
// group, so every wave executes one primitive with no divergence. The chain value lives
// in an n x 64-byte device buffer between the steps (one stream, no host round trip); the final
// hash is its first 32 bytes. A batch step is one x16r_step_all launch (grid y = slot); the nonce
// search, where every nonce of a window runs the same slot, launches that slot's own kernel
// (x16r_step_<slot>, its own register allocation) over the whole window. The primitives are hip/kernels/x16r_device.hpp (the host's
// constructions, tables generated from them).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_params.h"

#define X16R_FN __device__ inline
#include "x16r_device.hpp"

#define X16R_BLOCK 64

// One (step, slot) group: slot A is a template parameter, so each slot is its own kernel with its
// own register allocation (the light ARX slots are not held to the occupancy of the heaviest).
// The slot's lookup tables copied into LDS once per workgroup (the per-lane byte-indexed lookups
// would otherwise be 64 scattered global loads per instruction): Groestl's and Whirlpool's 8 x 256
// u64, Fugue's 4 x 256 u32, the AES round tables (4 x 256 u32) of SHAvite-3 and ECHO, and Tiger's 4 x 256 u64 on the
// slots X16RV2 pre-hashes with it.
template <typename T, int N>
__device__ void x16r_stage(T* dst, const T* src) {
    for (int i = threadIdx.x; i < N; i += X16R_BLOCK) dst[i] = src[i];
}

// LDS bytes slot A uses (its tables and, for SIMD, the lanes' NTT buffers); a slot uses one region.
template <int A>
constexpr int x16r_lds_bytes() {
    return (A == 2 || A == 14) ? 16384 : (A == 4 || A == 6 || A == 15) ? 8192 : (A == 8 || A == 10 || A == 12) ? 4096
         : A == 9 ? 2 * (256 * X16R_BLOCK + 768) : 8;
}
#define X16R_LDS_MAX_BYTES (2 * (256 * X16R_BLOCK + 768))

template <int A>
__device__ void x16r_group(const X16rStepParams& p, uint64_t* lds) {
    constexpr bool kGroestl = A == 2, kWhirl = A == 14, kFugue = A == 12, kAes = A == 8 || A == 10;
    constexpr bool kTiger = A == 4 || A == 6 || A == 15;
    uint64_t* t64 = lds;                                // Groestl / Whirlpool / Tiger tables
    uint32_t* t32 = (uint32_t*)lds;                     // Fugue / AES tables
    int16_t* ntt = (int16_t*)lds;                       // SIMD: each lane's NTT buffer, lanes interleaved
    int16_t* simd_t = ntt + 256 * X16R_BLOCK;           // SIMD: 41^k mod 257 and the two y offsets
    if (kGroestl) x16r_stage<uint64_t, 2048>(t64, kX16rGroestlT);
    if (kWhirl) x16r_stage<uint64_t, 2048>(t64, kX16rWhirlT);
    if (kTiger) x16r_stage<uint64_t, 1024>(t64, kX16rTiger);
    if (kFugue) x16r_stage<uint32_t, 1024>(t32, kX16rFugueMt);
    if (kAes) x16r_stage<uint32_t, 1024>(t32, kX16rAesT);
    if (A == 9) {
        x16r_stage<int16_t, 256>(simd_t, kX16rSimdPw);
        x16r_stage<int16_t, 256>(simd_t + 256, kX16rSimdYn);
        x16r_stage<int16_t, 256>(simd_t + 512, kX16rSimdYf);
    }
    if (kGroestl || kWhirl || kTiger || kFugue || kAes || A == 9) __syncthreads();  // every thread, before any exits

    const int32_t lo = p.offsets[A], hi = p.offsets[A + 1];
    const int32_t k = lo + (int32_t)(blockIdx.x * X16R_BLOCK + threadIdx.x);
    if (k >= hi) return;
    const uint32_t i = (uint32_t)p.order[k];
    if (i >= p.n) return;
    uint8_t in[80];
    const int len = p.step == 0 ? 80 : 64;
    const bool search = p.tmpl != nullptr;
    const uint4* src = (const uint4*)(p.step != 0 ? p.state + (size_t)i * 64 : search ? p.tmpl : p.headers + (size_t)i * 80);
    for (int w = 0; w < len / 16; ++w) {
        const uint4 v = src[w];
        x16rd::st32(in + 16 * w, v.x);
        x16rd::st32(in + 16 * w + 4, v.y);
        x16rd::st32(in + 16 * w + 8, v.z);
        x16rd::st32(in + 16 * w + 12, v.w);
    }
    if (search && p.step == 0) x16rd::st32(in + 76, p.start_nonce + i);
    const bool v2 = search ? p.v2_all != 0 : p.v2[i] != 0;
    uint8_t out[64];
    if (kTiger && v2) {  // X16RV2: Tiger-192 first
        uint8_t t[64];
        x16rd::tiger192_padded(in, len, t, t64);
        x16rd::single(A, t, 64, out);
    } else if (kGroestl) {
        x16rd::groestl512(in, len, out, t64);
    } else if (kWhirl) {
        x16rd::whirlpool512(in, len, out, t64);
    } else if (kFugue) {
        x16rd::fugue512(in, len, out, t32);
    } else if (A == 9) {
        x16rd::simd512(in, len, out, ntt + threadIdx.x, X16R_BLOCK, simd_t, simd_t + 256, simd_t + 512);
    } else if (A == 8) {
        x16rd::shavite512(in, len, out, t32);
    } else if (A == 10) {
        x16rd::echo512(in, len, out, t32);
    } else {
        x16rd::single(A, in, len, out);
    }
    uint4* dst = (uint4*)(p.state + (size_t)i * 64);
    for (int w = 0; w < 4; ++w)
        dst[w] = make_uint4(x16rd::ld32(out + 16 * w), x16rd::ld32(out + 16 * w + 4), x16rd::ld32(out + 16 * w + 8),
                            x16rd::ld32(out + 16 * w + 12));
}

extern "C" __global__ __launch_bounds__(256) void x16r_hits(X16rHitParams p) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.n) return;
    const uint4* h = (const uint4*)(p.state + (size_t)i * 64);
    const uint4 lo = h[0], hi = h[1];
    const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    bool le = true;
    for (int k = 7; k >= 0; --k) {
        if (w[k] != p.target[k]) {
            le = w[k] < p.target[k];
            break;
        }
    }
    if (le) atomicMin(p.best, i);
}

#define X16R_SLOT(A)                                                                         \
    extern "C" __global__ __launch_bounds__(X16R_BLOCK) void x16r_step_##A(X16rStepParams p) {     \
        __shared__ uint64_t lds[x16r_lds_bytes<A>() / 8];                                        \
        [[clang::always_inline]] x16r_group<A>(p, lds);                                          \
    }
X16R_SLOT(0) X16R_SLOT(1) X16R_SLOT(2) X16R_SLOT(3) X16R_SLOT(4) X16R_SLOT(5) X16R_SLOT(6) X16R_SLOT(7)
X16R_SLOT(8) X16R_SLOT(9) X16R_SLOT(10) X16R_SLOT(11) X16R_SLOT(12) X16R_SLOT(13) X16R_SLOT(14) X16R_SLOT(15)

// Every slot group of a step in ONE launch (grid y = slot, each workgroup's slot uniform): the 16
// groups run side by side, at the cost of one register allocation (the heaviest slot's) for all of
// them -- 2.27 M against 1.91 M hashes/s for per-slot launches on 4 streams (profiles r5k).
extern "C" __global__ __launch_bounds__(X16R_BLOCK) void x16r_step_all(X16rStepParams p) {
    __shared__ uint64_t lds[X16R_LDS_MAX_BYTES / 8];
    switch (blockIdx.y) {
        case 0: x16r_group<0>(p, lds); break;
        case 1: x16r_group<1>(p, lds); break;
        case 2: x16r_group<2>(p, lds); break;
        case 3: x16r_group<3>(p, lds); break;
        case 4: x16r_group<4>(p, lds); break;
        case 5: x16r_group<5>(p, lds); break;
        case 6: x16r_group<6>(p, lds); break;
        case 7: x16r_group<7>(p, lds); break;
        case 8: x16r_group<8>(p, lds); break;
        case 9: [[clang::always_inline]] x16r_group<9>(p, lds); break;  // SIMD: too big for the inliner's budget
        case 10: x16r_group<10>(p, lds); break;
        case 11: x16r_group<11>(p, lds); break;
        case 12: x16r_group<12>(p, lds); break;
        case 13: x16r_group<13>(p, lds); break;
        case 14: x16r_group<14>(p, lds); break;
        default: x16r_group<15>(p, lds); break;
    }
}
