// DAG build probe on one MI355X (gfx950): what bounds `ethash_dag_build`, and the thread-per-item
// layout it replaced against the quad-per-item layout it ships.
//
// Every 512-bit DAG item is 512 dependent 64-byte parent reads from the light cache (16 MiB at
// epoch 0 .. 64 MiB at epoch 384, resident in the 256 MiB Infinity Cache; the reference's
// src/crypto/ethash/lib/ethash/ethash.cpp:180-207). The thread form gives each thread one item
// and reads a parent as four 16-byte loads (four wave-wide loads touching 64 lines each). The
// quad form gives each item four lanes: one 16-byte load per lane per parent (one wave-wide load
// touching 16 lines, each read whole by its quad), the parent index word broadcast in the quad by
// DPP. Both read exactly the same bytes; the quad form issues a quarter of the load instructions.
//
//   ceil-thread / ceil-quad : the same loads with independent (hashed) indices, no fnv chain: the
//                             memory system's rate for random 64-byte reads of a light-cache-sized
//                             buffer, in each layout
//   ship                    : hip/kernels/ethash_dag.hip as built into the engine (quad, 1 item)
//   thread                  : the round-1..6 engine kernel (one item per thread), kept here
//   quad-N                  : quad per item, N items per quad interleaved (N chains in flight)
// Every other variant's output is compared byte for byte with ship's over the same items.
// r6m (before the switch, ship = thread): ceil-quad 3.68 TB/s, thread 3.46, quad-1 3.80 at
// epoch 384; 5.16 / 4.73 / 5.17 at epoch 0; quad-2 / quad-4 no better than quad-1.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/dag_build_probe tools/dag_build_probe.hip
//   tools/bin/dag_build_probe [light_items]
#include "../nodexa_chain_core_amd/hip/kernels/ethash_dag.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

NX_DEV uint32_t pb_mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

template <int C>
NX_DEV uint32_t pb_qb(uint32_t v) {  // lane C of each aligned quad, to the whole quad
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, C * 0x55, 0xf, 0xf, false);
}

NX_DEV uint32_t pb_mod(uint32_t x, const FastMod32& f) {  // Barrett, one correction
    const uint32_t r = x - __umulhi(x, f.mb) * f.d;
    return min(r, r - f.d);
}

// ---- ceilings: 512 parent reads per item, indices hashed (no dependency on the data)
__global__ __launch_bounds__(256) void ceil_thread(EthashDagParams p, FastMod32 lmod, uint32_t* out) {
    const uint64_t item = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (item >= p.num_items) return;
    const uint4* light = (const uint4*)p.light;
    uint32_t acc = 0, h = (uint32_t)item * 0x9e3779b9u;
#pragma unroll 1
    for (uint32_t j = 0; j < 512; j += 16) {
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t parent = pb_mod(pb_mix32(h + j + k), lmod);
            const uint4* src = light + (size_t)parent * 4;
            const uint4 a = src[0], b = src[1], c = src[2], d = src[3];
            acc += (a.x ^ a.y ^ a.z ^ a.w) + (b.x ^ b.y ^ b.z ^ b.w) + (c.x ^ c.y ^ c.z ^ c.w) + (d.x ^ d.y ^ d.z ^ d.w);
        }
    }
    if (acc == 0x12345678u) out[item] = acc;
}

__global__ __launch_bounds__(256) void ceil_quad(EthashDagParams p, FastMod32 lmod, uint32_t* out) {
    const uint64_t item = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 2;
    const uint32_t s = threadIdx.x & 3;
    if (item >= p.num_items) return;
    const uint4* light = (const uint4*)p.light;
    uint32_t acc = 0, h = (uint32_t)item * 0x9e3779b9u;
#pragma unroll 1
    for (uint32_t j = 0; j < 512; j += 16) {
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t parent = pb_mod(pb_mix32(h + j + k), lmod);
            const uint4 v = light[(size_t)parent * 4 + s];
            acc += v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) out[item] = acc;
}

// ---- thread per item (the engine's kernel through round 6)
__global__ __launch_bounds__(256) void dag_thread(EthashDagParams p, FastMod32 lmod) {
    const uint64_t local = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (local >= p.num_items) return;
    const uint64_t index = p.first_item + local;
    const uint4* __restrict__ light = (const uint4*)p.light;
    const uint32_t seed = (uint32_t)index;
    uint32_t mix[16];
    {
        const uint32_t li = pb_mod(seed, lmod);
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
            const uint32_t parent = pb_mod(fnv1(seed ^ (j + k), mix[k]), lmod);
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
    uint4* dst = (uint4*)p.dag + (size_t)index * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        dst[k] = make_uint4((uint32_t)out[2 * k], (uint32_t)(out[2 * k] >> 32), (uint32_t)out[2 * k + 1],
                            (uint32_t)(out[2 * k + 1] >> 32));
}

// ---- quad per item, N items per quad: lane s of the quad owns words 4s..4s+3 of each item's mix
template <int N>
__global__ __launch_bounds__(256) void dag_quad(EthashDagParams p, FastMod32 lmod) {
    const uint64_t quad = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 2;
    const uint32_t s = threadIdx.x & 3;
    const uint4* __restrict__ light = (const uint4*)p.light;
    uint32_t seed[N];
    uint32_t m[N][4];
#pragma unroll
    for (int t = 0; t < N; ++t) {
        uint64_t local = quad * N + t;
        local = local < p.num_items ? local : p.num_items - 1;  // tail quads recompute the last item
        seed[t] = (uint32_t)(p.first_item + local);
        const uint32_t li = pb_mod(seed[t], lmod);
        uint64_t in[8], o[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v = light[(size_t)li * 4 + k];
            in[2 * k] = ((uint64_t)v.y << 32) | v.x;
            in[2 * k + 1] = ((uint64_t)v.w << 32) | v.z;
        }
        in[0] ^= seed[t];
        keccak512_64(in, o);
        const uint64_t lo = (s & 2) ? ((s & 1) ? o[6] : o[4]) : ((s & 1) ? o[2] : o[0]);
        const uint64_t hi = (s & 2) ? ((s & 1) ? o[7] : o[5]) : ((s & 1) ? o[3] : o[1]);
        m[t][0] = (uint32_t)lo; m[t][1] = (uint32_t)(lo >> 32);
        m[t][2] = (uint32_t)hi; m[t][3] = (uint32_t)(hi >> 32);
    }
#pragma unroll 1
    for (uint32_t j = 0; j < 512; j += 16) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            uint4 v[N];
#pragma unroll
            for (int t = 0; t < N; ++t) {
                const uint32_t own = m[t][k & 3];
                uint32_t mk;
                switch (k >> 2) {
                    case 0: mk = pb_qb<0>(own); break;
                    case 1: mk = pb_qb<1>(own); break;
                    case 2: mk = pb_qb<2>(own); break;
                    default: mk = pb_qb<3>(own); break;
                }
                const uint32_t parent = pb_mod(fnv1(seed[t] ^ (j + (uint32_t)k), mk), lmod);
                v[t] = light[(size_t)parent * 4 + s];
            }
#pragma unroll
            for (int t = 0; t < N; ++t) {
                m[t][0] = fnv1(m[t][0], v[t].x); m[t][1] = fnv1(m[t][1], v[t].y);
                m[t][2] = fnv1(m[t][2], v[t].z); m[t][3] = fnv1(m[t][3], v[t].w);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < N; ++t) {
        uint32_t all[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            all[k] = pb_qb<0>(m[t][k]);
            all[4 + k] = pb_qb<1>(m[t][k]);
            all[8 + k] = pb_qb<2>(m[t][k]);
            all[12 + k] = pb_qb<3>(m[t][k]);
        }
        uint64_t in[8], o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) in[k] = ((uint64_t)all[2 * k + 1] << 32) | all[2 * k];
        keccak512_64(in, o);
        const uint64_t local = quad * N + t;
        if (local < p.num_items) {
            const uint64_t lo = (s & 2) ? ((s & 1) ? o[6] : o[4]) : ((s & 1) ? o[2] : o[0]);
            const uint64_t hi = (s & 2) ? ((s & 1) ? o[7] : o[5]) : ((s & 1) ? o[3] : o[1]);
            ((uint4*)p.dag)[(p.first_item + local) * 4 + s] =
                make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
        }
    }
}

__global__ void fill(uint4* a, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t x = pb_mix32(uint32_t(i) * 4 + 1), y = pb_mix32(x ^ 0x51ed270bu);
        a[i] = make_uint4(x, y, x ^ 0x9e3779b9u, y + 0x85ebca6bu);
    }
}

static FastMod32 make_mod(uint32_t d) {
    uint32_t s = 0;
    while ((uint64_t(1) << s) < d) ++s;
    FastMod32 f{};
    f.d = d;
    f.m = uint32_t(((uint64_t(1) << 32) * ((uint64_t(1) << s) - d)) / d + 1);
    f.s = s;
    f.mb = uint32_t((uint64_t(1) << 32) / d);
    return f;
}

template <class L>
static float time_best(L launch) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch();  // warm
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(a));
        launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return best;
}

static void report(const char* name, uint64_t items, float ms, long mismatches) {
    // bytes the kernel reads: 512 parents x 64 B per item (the 64 B seed read and the store aside)
    const double tb = double(items) * 512 * 64 / (ms * 1e-3) / 1e12;
    std::printf("{\"variant\":\"%s\",\"items\":%llu,\"ms\":%.3f,\"m_items_s\":%.1f,\"parent_tb_s\":%.3f,"
                "\"full_dag_4gib_s\":%.3f,\"mismatched_items\":%ld}\n",
                name, (unsigned long long)items, ms, items / (ms * 1e3), tb, ms * 1e-3 * (67108864.0 / items),
                mismatches);
    std::fflush(stdout);
}

int main(int argc, char** argv) {
    // epoch 384's light cache: 1,048,571 items of 64 B (any nearby count prices the same)
    const uint32_t light_items = argc > 1 ? uint32_t(std::strtoul(argv[1], nullptr, 0)) : 1048571u;
    const uint64_t items = 1ull << 22;  // one engine launch (ops/ethash._DAG_CHUNK)
    uint4 *light = nullptr, *dag = nullptr, *dag2 = nullptr;
    uint32_t* sink = nullptr;
    CHECK(hipMalloc(&light, size_t(light_items) * 64));
    CHECK(hipMalloc(&dag, items * 64));
    CHECK(hipMalloc(&dag2, items * 64));
    CHECK(hipMalloc(&sink, items * 4));
    fill<<<4096, 256>>>(light, size_t(light_items) * 4);
    CHECK(hipDeviceSynchronize());
    const FastMod32 lmod = make_mod(light_items);
    EthashDagParams p{};
    p.light = light;
    p.first_item = 0;
    p.num_items = items;
    p.light_items = light_items;
    std::printf("{\"light_items\":%u,\"light_mib\":%.1f}\n", light_items, light_items * 64.0 / (1 << 20));

    report("ceil-thread", items, time_best([&] { ceil_thread<<<unsigned(items / 256), 256>>>(p, lmod, sink); }), -1);
    report("ceil-quad", items, time_best([&] { ceil_quad<<<unsigned(items * 4 / 256), 256>>>(p, lmod, sink); }), -1);

    p.dag = dag;
    report("ship", items, time_best([&] { ethash_dag_build<<<unsigned(items / 64), 256>>>(p, lmod); }), -1);
    std::vector<uint8_t> ref(items * 64), got(items * 64);
    CHECK(hipMemcpy(ref.data(), dag, items * 64, hipMemcpyDeviceToHost));
    auto check = [&](const char* name, float ms) {
        CHECK(hipMemcpy(got.data(), dag2, items * 64, hipMemcpyDeviceToHost));
        long bad = 0;
        for (uint64_t i = 0; i < items; ++i) bad += std::memcmp(&ref[i * 64], &got[i * 64], 64) != 0;
        report(name, items, ms, bad);
    };
    p.dag = dag2;
    CHECK(hipMemset(dag2, 0, items * 64));
    check("thread", time_best([&] { dag_thread<<<unsigned(items / 256), 256>>>(p, lmod); }));
    CHECK(hipMemset(dag2, 0, items * 64));
    check("quad-2", time_best([&] { dag_quad<2><<<unsigned(items * 4 / 2 / 256), 256>>>(p, lmod); }));
    CHECK(hipMemset(dag2, 0, items * 64));
    check("quad-4", time_best([&] { dag_quad<4><<<unsigned(items * 4 / 4 / 256), 256>>>(p, lmod); }));
    CHECK(hipFree(light));
    CHECK(hipFree(dag));
    CHECK(hipFree(dag2));
    CHECK(hipFree(sink));
    return 0;
}
