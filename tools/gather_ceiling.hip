// Random 256-byte row gather ceiling on one MI355X (the KawPow DAG access pattern).
//
// KawPow reads one 256 B DAG row per round per hash, 64 rounds, and the next row's
// index depends on the row just read (src/crypto/ethash/lib/ethash/progpow.cpp:182-184,
// 227-244). This program measures what the memory system gives that pattern with no
// ProgPoW arithmetic around it, so the search kernel's MH/s can be priced against a
// measured ceiling instead of the 8 TB/s datasheet figure:
//   dep   : 16-lane group = one chain, next index from the row just loaded (KawPow shape)
//   indep : indices from a hash of (nonce, round): no dependency, pure gather bandwidth
// CH chains are interleaved per group (more rows in flight per wave).
//
//   hipcc --offload-arch=gfx950 -O3 -o gather_ceiling tools/gather_ceiling.hip && ./gather_ceiling
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int CH, bool DEP, bool NT, int BLOCK, int LDS_WORDS>
__global__ __launch_bounds__(BLOCK) void gather(const uint4* __restrict__ rows, uint32_t nrows,
                                                uint32_t* __restrict__ out, uint32_t seed) {
    __shared__ uint32_t pad[LDS_WORDS > 0 ? LDS_WORDS : 1];
    if (LDS_WORDS > 0) {  // occupy LDS like the search kernel's L1 table (workgroups per CU)
        pad[threadIdx.x % (LDS_WORDS > 0 ? LDS_WORDS : 1)] = threadIdx.x;
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 15;
    const uint32_t gid = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t acc = LDS_WORDS > 0 ? pad[(threadIdx.x * 7) % (LDS_WORDS > 0 ? LDS_WORDS : 1)] : 0;
#pragma unroll 1
    for (int h = 0; h < 16; h += CH) {
        uint32_t x[CH];
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = mix32(seed ^ (gid * 16 + h + c));
#pragma unroll 1
        for (uint32_t r = 0; r < 64; ++r) {
            uint4 d[CH];
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                uint32_t key = DEP ? __shfl(x[c], int(r & 15), 16) : mix32(x[c] + r);
                if (!DEP) key = __shfl(key, 0, 16);
                const uint32_t idx = key % nrows;
                const uint4* p = rows + (size_t)idx * 16 + (lane ^ (r & 15));
                if (NT) {
                    const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
                    d[c] = make_uint4(v.x, v.y, v.z, v.w);
                } else {
                    d[c] = *p;
                }
            }
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                if (DEP)
                    x[c] = (x[c] ^ d[c].x) * 33u + (d[c].y ^ d[c].z ^ d[c].w);
                else
                    acc += d[c].x ^ d[c].y ^ d[c].z ^ d[c].w;
            }
        }
#pragma unroll
        for (int c = 0; c < CH; ++c) acc ^= x[c];
    }
    if (acc == 0x12345678u) out[gid] = acc;  // keep the loads alive
}

__global__ void fill(uint4* rows, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t a = mix32(uint32_t(i)), b = mix32(uint32_t(i >> 32) ^ a);
        rows[i] = make_uint4(a, b, a ^ 0x9e3779b9u, b + 0x85ebca6bu);
    }
}

template <int CH, bool DEP, bool NT, int BLOCK, int LDS_WORDS>
static void run(const char* name, const uint4* rows, uint32_t nrows, uint32_t* out, uint64_t nonces) {
    const unsigned grid = unsigned(nonces / BLOCK);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    gather<CH, DEP, NT, BLOCK, LDS_WORDS><<<grid, BLOCK>>>(rows, nrows, out, 1);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(a));
        gather<CH, DEP, NT, BLOCK, LDS_WORDS><<<grid, BLOCK>>>(rows, nrows, out, 2 + rep);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    const double bytes = double(grid) * BLOCK * 64.0 * 256.0;  // every nonce = one 64-round chain
    std::printf("{\"variant\":\"%s\",\"chains\":%d,\"dep\":%d,\"nt\":%d,\"block\":%d,\"lds_kib\":%d,"
                "\"ms\":%.3f,\"tb_s\":%.3f,\"mchains_s\":%.1f}\n",
                name, CH, int(DEP), int(NT), BLOCK, LDS_WORDS / 256, best, bytes / best / 1e9,
                double(grid) * BLOCK / best / 1e3);
    std::fflush(stdout);
}

int main() {
    // epoch-384 DAG: 16,777,213 rows of 256 B (4.00 GiB); any nearby row count prices the same
    const uint32_t nrows = 16777213u;
    const size_t bytes = size_t(nrows) * 256;
    uint4* rows = nullptr;
    uint32_t* out = nullptr;
    CHECK(hipMalloc(&rows, bytes));
    CHECK(hipMalloc(&out, sizeof(uint32_t) << 26));
    fill<<<4096, 256>>>(rows, bytes / 16);
    CHECK(hipDeviceSynchronize());
    const uint64_t n = 1ull << 24;  // nonces per launch
    run<1, true, true, 768, 16384>("dep-kawpow-shape", rows, nrows, out, n);
    run<1, true, false, 768, 16384>("dep-kawpow-shape-cached", rows, nrows, out, n);
    run<1, true, true, 1024, 0>("dep-32waves", rows, nrows, out, n);
    run<2, true, true, 1024, 0>("dep-2ch", rows, nrows, out, n);
    run<4, true, true, 1024, 0>("dep-4ch", rows, nrows, out, n);
    run<2, true, true, 768, 16384>("dep-2ch-kawpow-occ", rows, nrows, out, n);
    run<4, false, true, 1024, 0>("indep-4ch", rows, nrows, out, n);
    run<4, false, false, 1024, 0>("indep-4ch-cached", rows, nrows, out, n);
    run<8, false, true, 1024, 0>("indep-8ch", rows, nrows, out, n);
    CHECK(hipFree(rows));
    CHECK(hipFree(out));
    return 0;
}
