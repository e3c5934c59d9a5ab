// Random row scatter ceiling on one MI355X (the Equihash row-emission pattern).
//
// Every Wagner round appends ~2M rows per instance to random buckets (equihash_ps.hip). This
// program prices that store pattern with nothing around it: each group of G lanes writes one
// run of G * S contiguous bytes (S per lane) at a random run-aligned offset of a 4 GiB buffer.
// G = 1 is Equihash's one row per lane; G > 1 shows what a write-combined (bucket-major) layout
// would get for the same bytes. NT = nontemporal stores.
//
//   hipcc --offload-arch=gfx950 -O3 -o scatter_ceiling tools/scatter_ceiling.hip && ./scatter_ceiling [a|m|c]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int PER = 16;  // rows per lane per launch

template <int S, int G, bool NT>
__global__ __launch_bounds__(256) void scatter(uint32_t* __restrict__ buf, uint32_t nruns, uint32_t seed) {
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    const uint32_t grp = gid / G, lane = gid % G;
#pragma unroll 1
    for (int k = 0; k < PER; ++k) {
        const uint32_t run = mix32(seed ^ (grp * PER + k)) % nruns;
        uint32_t* dst = buf + ((size_t)run * G * S + (size_t)lane * S) / 4;
        const uint32_t v = gid ^ k;
#pragma unroll
        for (int q = 0; q < S / 16; ++q) {
            const u32x4 w = {v, v + 1, v + 2, (uint32_t)q};
            if (NT)
                __builtin_nontemporal_store(w, (u32x4*)dst + q);
            else
                ((u32x4*)dst)[q] = w;
        }
        if constexpr (S % 16 == 8) {
            uint2* d2 = (uint2*)(dst + (S / 16) * 4);
            *d2 = make_uint2(v, k);
        }
        if constexpr (S % 16 == 4) dst[(S / 16) * 4] = v;
    }
}

// L2 write merging probe: rows written by DIFFERENT store instructions (other lanes, waves and
// workgroups) into the same 128-byte lines. Workgroup b writes its 256 x PER rows of S bytes at
// random row positions of region r(b); BPR workgroups share a region of BPR * 256 * PER rows, so
// each line is filled by ~128/S stores from as many workgroups, close together in time. XCD = 1:
// only workgroups of one XCD share a region (b and b + 8 share an XCD); XCD = 0: consecutive
// workgroups (eight XCDs) share it. EA write requests per row ~1 mean no merging in L2.
template <int S, bool XCD>
__global__ __launch_bounds__(256) void l2merge(uint32_t* __restrict__ buf, uint32_t bpr, uint32_t nreg, uint32_t seed) {
    const uint32_t b = blockIdx.x;
    const uint32_t reg = (XCD ? (b % 8) * (gridDim.x / 8 / bpr) + (b / 8) / bpr : b / bpr) % nreg;
    const uint32_t rrows = bpr * 256 * PER;
    const uint32_t gid = b * 256 + threadIdx.x;
#pragma unroll 1
    for (int k = 0; k < PER; ++k) {
        const uint32_t row = mix32(seed ^ (gid * PER + k)) % rrows;
        u32x4* dst = (u32x4*)(buf + ((size_t)reg * rrows + row) * (S / 4));
#pragma unroll
        for (int q = 0; q < S / 16; ++q) dst[q] = u32x4{gid, (uint32_t)k, seed, (uint32_t)q};
    }
}

// Random row gathers: each lane reads PER rows of S bytes at random row positions of a `bytes`
// working set (the price of a layout that moves the scatter to the next round's reads).
template <int S>
__global__ __launch_bounds__(256) void gather(const uint32_t* __restrict__ buf, uint32_t nrows, uint32_t seed,
                                              uint32_t* __restrict__ sink) {
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    uint32_t acc = 0;
    u32x4 v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const uint32_t row = mix32(seed ^ (gid * PER + k)) % nrows;
        v[k] = ((const u32x4*)(buf + (size_t)row * (S / 4)))[0];
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) acc ^= v[k].x + v[k].y + v[k].z + v[k].w;
    if (acc == 0x12345678u) sink[0] = gid;
}

// Equihash-shaped append probe: 256 workgroups of 1024 threads = 16 instances x 16 writers, each
// thread appending ROWS_PER_THREAD rows of S bytes to random buckets of its instance (4096 buckets,
// 2^21 rows per instance, 512 per bucket on average). GLOBAL = 0: the private-slot scheme of
// equihash_ps.hip (LDS slot counters, writer-private segments of SEG slots in every bucket);
// GLOBAL = 1: one returning global atomic per row on the instance's bucket counter, so the rows
// of all writers of a bucket land next to each other. XCD = 1 puts all 16 writers of an instance
// on one XCD (instance = workgroup id mod 16), so with GLOBAL = 1 a bucket's tail line is written
// by one L2 only.
constexpr uint32_t AP_BUCKETS = 4096, AP_INST = 16, AP_WRITERS = 16, AP_SEG = 48, AP_CAP = AP_WRITERS * AP_SEG;
constexpr int ROWS_PER_THREAD = 128;

template <int S, bool GLOBAL, bool XCD>
__global__ __launch_bounds__(1024) void append_probe(uint32_t* __restrict__ buf, uint32_t* __restrict__ gcnt,
                                                     uint32_t seed, uint32_t* __restrict__ dropped) {
    __shared__ uint32_t cnt2[AP_BUCKETS / 2];
    const uint32_t lin = blockIdx.x;
    const uint32_t inst = XCD ? lin % AP_INST : lin / AP_WRITERS, grp = XCD ? lin / AP_INST : lin % AP_WRITERS;
    if (!GLOBAL) {
        for (uint32_t k = threadIdx.x; k < AP_BUCKETS / 2; k += 1024) cnt2[k] = 0;
        __syncthreads();
    }
    const uint32_t gid = lin * 1024 + threadIdx.x;
    uint32_t drop = 0;
#pragma unroll 1
    for (int k = 0; k < ROWS_PER_THREAD; ++k) {
        const uint32_t b = mix32(seed ^ (gid * ROWS_PER_THREAD + k)) % AP_BUCKETS;
        size_t row;
        if (GLOBAL) {
            const uint32_t slot = atomicAdd(&gcnt[inst * AP_BUCKETS + b], 1u);
            if (slot >= AP_CAP) { ++drop; continue; }
            row = ((size_t)inst * AP_BUCKETS + b) * AP_CAP + slot;
        } else {
            const uint32_t sh = (b & 1u) << 4;
            const uint32_t slot = (atomicAdd(&cnt2[b >> 1], 1u << sh) >> sh) & 0xFFFFu;
            if (slot >= AP_SEG) { ++drop; continue; }
            row = ((size_t)inst * AP_BUCKETS + b) * AP_CAP + grp * AP_SEG + slot;
        }
        uint32_t* dst = buf + row * (S / 4);
#pragma unroll
        for (int q = 0; q < S / 4; ++q) dst[q] = gid ^ (uint32_t)(k + q);
    }
    if (drop) atomicAdd(dropped, drop);
}

template <int S, bool GLOBAL, bool XCD>
static void run_append(const char* name, uint32_t* buf, uint32_t* gcnt, uint32_t* dropped) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        CHECK(hipMemset(gcnt, 0, AP_INST * AP_BUCKETS * 4));
        CHECK(hipMemset(dropped, 0, 4));
        CHECK(hipEventRecord(a));
        append_probe<S, GLOBAL, XCD><<<AP_INST * AP_WRITERS, 1024>>>(buf, gcnt, 7 + rep, dropped);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (rep) best = ms < best ? ms : best;  // rep 0 warms
    }
    uint32_t d = 0;
    CHECK(hipMemcpy(&d, dropped, 4, hipMemcpyDeviceToHost));
    const double rows = double(AP_INST) * AP_WRITERS * 1024 * ROWS_PER_THREAD;
    std::printf("{\"variant\":\"%s\",\"row_bytes\":%d,\"global_atomic\":%d,\"xcd_local\":%d,\"ms\":%.3f,"
                "\"grows_s\":%.2f,\"dropped\":%u}\n",
                name, S, int(GLOBAL), int(XCD), best, rows / best / 1e6, d);
    std::fflush(stdout);
}

template <int S, int G, bool NT>
static void run(const char* name, uint32_t* buf, size_t bytes, uint64_t lanes) {
    const uint32_t nruns = uint32_t(bytes / (size_t(G) * S));
    const unsigned grid = unsigned(lanes / 256);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    scatter<S, G, NT><<<grid, 256>>>(buf, nruns, 1);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(a));
        scatter<S, G, NT><<<grid, 256>>>(buf, nruns, 2 + rep);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    const double rows = double(grid) * 256 * PER;
    std::printf("{\"variant\":\"%s\",\"row_bytes\":%d,\"run_lanes\":%d,\"nt\":%d,\"target_mib\":%zu,\"ms\":%.3f,"
                "\"tb_s\":%.3f,\"grows_s\":%.2f}\n",
                name, S, G, int(NT), bytes >> 20, best, rows * S / best / 1e9, rows / best / 1e6);
    std::fflush(stdout);
}

template <int S, bool XCD>
static void run_merge(const char* name, uint32_t* buf, size_t bytes, uint32_t bpr) {
    const unsigned grid = 16384;  // 4M lanes x PER = 64M rows
    const uint32_t rrows = bpr * 256 * PER;
    const uint32_t nreg = uint32_t(bytes / (size_t(rrows) * S));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    l2merge<S, XCD><<<grid, 256>>>(buf, bpr, nreg, 1);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(a));
        l2merge<S, XCD><<<grid, 256>>>(buf, bpr, nreg, 2 + rep);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    const double rows = double(grid) * 256 * PER;
    std::printf("{\"variant\":\"%s\",\"row_bytes\":%d,\"xcd_local\":%d,\"region_kib\":%u,\"ms\":%.3f,"
                "\"grows_s\":%.2f}\n",
                name, S, int(XCD), unsigned(size_t(rrows) * S / 1024), best, rows / best / 1e6);
    std::fflush(stdout);
}

template <int S>
static void run_gather(const char* name, uint32_t* buf, size_t ws, uint32_t* sink) {
    const unsigned grid = 16384;
    const uint32_t nrows = uint32_t(ws / S);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    gather<S><<<grid, 256>>>(buf, nrows, 1, sink);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(a));
        gather<S><<<grid, 256>>>(buf, nrows, 2 + rep, sink);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    const double rows = double(grid) * 256 * PER;
    std::printf("{\"variant\":\"%s\",\"row_bytes\":%d,\"ws_mib\":%u,\"ms\":%.3f,\"grows_s\":%.2f}\n", name, S,
                unsigned(ws >> 20), best, rows / best / 1e6);
    std::fflush(stdout);
}

int main(int argc, char** argv) {
    if (argc > 1 && argv[1][0] == 'a') {  // Equihash-shaped append probes (tools/gpu_r4v.sh)
        uint32_t *buf = nullptr, *gcnt = nullptr, *dropped = nullptr;
        const size_t bytes = size_t(AP_INST) * AP_BUCKETS * AP_CAP * 32;
        CHECK(hipMalloc(&buf, bytes));
        CHECK(hipMalloc(&gcnt, AP_INST * AP_BUCKETS * 4));
        CHECK(hipMalloc(&dropped, 4));
        CHECK(hipMemset(buf, 0, bytes));
        run_append<24, false, false>("private24", buf, gcnt, dropped);
        run_append<24, false, true>("private24-xcd", buf, gcnt, dropped);
        run_append<24, true, false>("global24", buf, gcnt, dropped);
        run_append<24, true, true>("global24-xcd", buf, gcnt, dropped);
        run_append<32, false, false>("private32", buf, gcnt, dropped);
        run_append<32, true, true>("global32-xcd", buf, gcnt, dropped);
        run_append<16, false, false>("private16", buf, gcnt, dropped);
        run_append<16, true, true>("global16-xcd", buf, gcnt, dropped);
        CHECK(hipFree(buf));
        CHECK(hipFree(gcnt));
        CHECK(hipFree(dropped));
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'c') {
        // Infinity Cache residency (round 6): the rounds' isolated-row stores into a target that
        // fits the 256 MB MALL against one that does not. 64M rows per launch at every size, so a
        // small target is rewritten many times (as a level's live rows would be by the next window)
        const size_t max_bytes = size_t(4) << 30;
        uint32_t* buf = nullptr;
        CHECK(hipMalloc(&buf, max_bytes));
        CHECK(hipMemset(buf, 0, max_bytes));
        const uint64_t lanes = 1ull << 22;
        for (size_t mib : {4096, 1024, 512, 256, 192, 128, 64, 32}) {
            const size_t bytes = mib << 20;
            run<16, 1, false>("row16", buf, bytes, lanes);
            run<24, 1, false>("row24", buf, bytes, lanes);
            run<32, 1, false>("row32", buf, bytes, lanes);
        }
        CHECK(hipFree(buf));
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'm') {  // merge + gather probes only (tools/gpu_r4t.sh)
        const size_t bytes = size_t(4) << 30;
        uint32_t *buf = nullptr, *sink = nullptr;
        CHECK(hipMalloc(&buf, bytes));
        CHECK(hipMalloc(&sink, 64));
        CHECK(hipMemset(buf, 0, bytes));
        run_merge<16, true>("merge16-xcd-bpr1", buf, bytes, 1);    // 64 KiB regions, one workgroup each
        run_merge<16, true>("merge16-xcd-bpr16", buf, bytes, 16);  // 1 MiB, 16 workgroups of one XCD
        run_merge<16, true>("merge16-xcd-bpr64", buf, bytes, 64);  // 4 MiB
        run_merge<16, false>("merge16-all-bpr16", buf, bytes, 16);  // 1 MiB shared by all XCDs
        run_merge<16, false>("merge16-all-bpr64", buf, bytes, 64);
        run_merge<32, true>("merge32-xcd-bpr16", buf, bytes, 16);
        run_gather<16>("gather16-4g", buf, bytes, sink);
        run_gather<16>("gather16-256m", buf, size_t(256) << 20, sink);
        run_gather<16>("gather16-64m", buf, size_t(64) << 20, sink);
        CHECK(hipFree(buf));
        CHECK(hipFree(sink));
        return 0;
    }
    const size_t bytes = size_t(4) << 30;
    uint32_t* buf = nullptr;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMemset(buf, 0, bytes));
    const uint64_t lanes = 1ull << 22;  // x PER rows = 64M rows per launch
    run<16, 1, false>("row16", buf, bytes, lanes);
    run<20, 1, false>("row20", buf, bytes, lanes);
    run<24, 1, false>("row24", buf, bytes, lanes);
    run<32, 1, false>("row32", buf, bytes, lanes);
    run<64, 1, false>("row64", buf, bytes, lanes);
    run<16, 1, true>("row16-nt", buf, bytes, lanes);
    run<32, 1, true>("row32-nt", buf, bytes, lanes);
    run<32, 2, false>("row32-run64", buf, bytes, lanes);
    run<32, 4, false>("row32-run128", buf, bytes, lanes);
    run<16, 8, false>("row16-run128", buf, bytes, lanes);
    run<32, 8, false>("row32-run256", buf, bytes, lanes);
    run<16, 4, false>("row16-run64", buf, bytes, lanes);
    CHECK(hipFree(buf));
    return 0;
}
