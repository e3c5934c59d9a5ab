// Equihash(200,9) round memory-pattern probe for a coarse-bucket / run-buffer layout (round 5).
//
// VERDICT r4 asks whether the rounds' one-EA-write-request-per-row floor (profiles/README r4r)
// can be beaten by (1) fewer destination buckets per level (D coarse buckets instead of 4096)
// with (2) a small LDS run buffer per destination that leaves the workgroup as one contiguous
// multi-row store when it fills, and (3) consumers that re-read a coarse bucket once per fine
// slice (K = fine / coarse reads of every row). This program prices (1)+(2) and (3) with nothing
// else around them, in the solver's shape: 256 workgroups of 1024 threads = 16 instances x 16
// writers, 2^21 rows per instance per level.
//
//   wr D RR S : every writer emits 2^17 rows of S bytes to uniformly random destinations d < D of
//               its instance, 576 rows (one per "consumer" thread) per batch. RR = 1: each row is
//               stored at its writer-private segment slot (the shipping scheme at D = 4096).
//               RR > 1: a row goes into the LDS run buffer of d; after each batch the full buffers
//               are flushed as RR contiguous rows of the segment; rows beyond RR in one batch go
//               straight to their slot. Two barriers per batch in every variant.
//   rd D K    : every workgroup streams the coarse buckets d = writer, writer + 16, ... of its
//               instance (all 16 writers' segments of each) K times over, as consumers of K fine
//               slices would (rows filtered, summed). Sequential: one workgroup reads its bucket K
//               times in a row (the re-reads should hit the L2 / MALL).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/eq_runs_probe tools/eq_runs_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

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

constexpr uint32_t INST = 16, WRITERS = 16, ROWS_PER_WRITER = 1u << 17, EMIT = 576;

// Segment capacity (rows) of one (instance, coarse bucket, writer): mean 2^17 / D, +8 sigma.
__host__ __device__ constexpr uint32_t seg_cap(uint32_t D) {
    return (ROWS_PER_WRITER / D) + 8 * (D >= 4096 ? 3u : D >= 1024 ? 6u : D >= 512 ? 8u : 12u) + 8;
}

template <int W>
struct __attribute__((aligned(4))) Row {
    uint32_t w[W];
};

template <uint32_t D, int RR, int W>
__global__ __launch_bounds__(1024) void wr(uint32_t* __restrict__ buf, uint32_t seed, uint32_t* __restrict__ dropped) {
    constexpr uint32_t CAP = seg_cap(D);
    constexpr int RB = RR > 1 ? RR : 1;
    __shared__ uint32_t segcnt[D];
    __shared__ uint32_t rcnt[RR > 1 ? D : 1];
    __shared__ uint32_t rbuf[RR > 1 ? D * RB * W : 1];
    const uint32_t inst = blockIdx.x / WRITERS, wtr = blockIdx.x % WRITERS;
    for (uint32_t k = threadIdx.x; k < D; k += 1024) {
        segcnt[k] = 0;
        if constexpr (RR > 1) rcnt[k] = 0;
    }
    __syncthreads();
    uint32_t drop = 0;
    auto seg_row = [&](uint32_t d, uint32_t slot) -> uint32_t* {
        return buf + ((((size_t)inst * D + d) * WRITERS + wtr) * CAP + slot) * W;
    };
    const uint32_t batches = ROWS_PER_WRITER / EMIT + 1;
#pragma unroll 1
    for (uint32_t bt = 0; bt < batches; ++bt) {
        const uint32_t idx = bt * EMIT + threadIdx.x;
        if (threadIdx.x < EMIT && idx < ROWS_PER_WRITER) {
            const uint32_t h = mix32(seed ^ (blockIdx.x * ROWS_PER_WRITER + idx));
            const uint32_t d = h % D;
            Row<W> r;
#pragma unroll
            for (int q = 0; q < W; ++q) r.w[q] = h + q;
            bool direct = true;
            if constexpr (RR > 1) {
                const uint32_t k = atomicAdd(&rcnt[d], 1u);
                if (k < RR) {
#pragma unroll
                    for (int q = 0; q < W; ++q) rbuf[(d * RB + k) * W + q] = r.w[q];
                    direct = false;
                }
            }
            if (direct) {
                const uint32_t slot = atomicAdd(&segcnt[d], 1u);
                if (slot < CAP) *(Row<W>*)seg_row(d, slot) = r; else ++drop;
            }
        }
        __syncthreads();
        if constexpr (RR > 1) {  // flush the full run buffers: RR contiguous rows each
            for (uint32_t d = threadIdx.x; d < D; d += 1024) {
                if (rcnt[d] >= RR) {
                    const uint32_t base = segcnt[d];
                    segcnt[d] = base + RR;
                    rcnt[d] = 0;
                    if (base + RR <= CAP) {
                        uint32_t* dst = seg_row(d, base);
#pragma unroll
                        for (int q = 0; q < RR * W; ++q) dst[q] = rbuf[d * RB * W + q];
                    } else {
                        drop += RR;
                    }
                }
            }
        }
        __syncthreads();
    }
    if constexpr (RR > 1) {  // the partial buffers at the end
        for (uint32_t d = threadIdx.x; d < D; d += 1024) {
            const uint32_t n = rcnt[d] < RR ? rcnt[d] : RR;
            const uint32_t base = segcnt[d];
            if (base + n <= CAP) {
                uint32_t* dst = seg_row(d, base);
                for (uint32_t q = 0; q < n * W; ++q) dst[q] = rbuf[d * RB * W + q];
            } else {
                drop += n;
            }
        }
    }
    if (drop) atomicAdd(dropped, drop);
}

// Consumer-side streaming: workgroup (inst, rdr) reads coarse buckets d = rdr, rdr + 16, ... of its
// instance K times each, every pass over the 16 writers' segments (fill = mean rows per segment).
template <uint32_t D, int W>
__global__ __launch_bounds__(1024) void rd(const uint32_t* __restrict__ buf, uint32_t K, uint32_t* __restrict__ sink) {
    constexpr uint32_t CAP = seg_cap(D), FILL = ROWS_PER_WRITER / D;
    const uint32_t inst = blockIdx.x / WRITERS, rdr = blockIdx.x % WRITERS;
    uint32_t acc = 0;
#pragma unroll 1
    for (uint32_t d = rdr; d < D; d += WRITERS) {
#pragma unroll 1
        for (uint32_t pass = 0; pass < K; ++pass) {
            // the bucket's 16 segments as one list of 16 * FILL rows
#pragma unroll 4
            for (uint32_t pos = threadIdx.x; pos < WRITERS * FILL; pos += 1024) {
                const uint32_t w = pos / FILL, s = pos % FILL;
                const Row<W> r = *(const Row<W>*)(buf + ((((size_t)inst * D + d) * WRITERS + w) * CAP + s) * W);
                acc += (r.w[0] >> 30) == pass % 4 ? r.w[W - 1] : 0u;  // the slice filter
            }
        }
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

static float time_ms(void (*launch)(void*), void* arg, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch(arg);  // warm
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a));
        launch(arg);
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

struct Ctx {
    uint32_t* buf;
    uint32_t* cnt;
    uint32_t seed;
    uint32_t K;
};

template <uint32_t D, int RR, int W>
static void launch_wr(void* p) {
    Ctx* c = (Ctx*)p;
    wr<D, RR, W><<<INST * WRITERS, 1024>>>(c->buf, c->seed++, c->cnt);
}

template <uint32_t D, int W>
static void launch_rd(void* p) {
    Ctx* c = (Ctx*)p;
    rd<D, W><<<INST * WRITERS, 1024>>>(c->buf, c->K, c->cnt);
}

template <uint32_t D, int RR, int W>
static void run_wr(Ctx& c) {
    CHECK(hipMemset(c.cnt, 0, 4));
    const float ms = time_ms(launch_wr<D, RR, W>, &c, 4);
    uint32_t dropped = 0;
    CHECK(hipMemcpy(&dropped, c.cnt, 4, hipMemcpyDeviceToHost));
    const double rows = double(INST) * WRITERS * ROWS_PER_WRITER;
    std::printf("{\"mode\":\"wr\",\"D\":%u,\"RR\":%d,\"row_bytes\":%d,\"ms\":%.4f,\"grows_s\":%.2f,\"dropped\":%u}\n", D, RR,
                4 * W, ms, rows / ms / 1e6, dropped);
    std::fflush(stdout);
}

template <uint32_t D, int W>
static void run_rd(Ctx& c, uint32_t K) {
    c.K = K;
    const float ms = time_ms(launch_rd<D, W>, &c, 4);
    const double rows = double(INST) * WRITERS * ROWS_PER_WRITER;  // rows per pass
    std::printf("{\"mode\":\"rd\",\"D\":%u,\"K\":%u,\"row_bytes\":%d,\"ms\":%.4f,\"ms_per_pass\":%.4f,\"tb_s\":%.3f}\n", D, K,
                4 * W, ms, ms / K, rows * K * 4 * W / ms / 1e9);
    std::fflush(stdout);
}

int main(int argc, char** argv) {
    const char* only = argc > 1 ? argv[1] : "all";
    Ctx c{};
    size_t bytes = 0;  // the largest layout of any variant below (D = 4096 .. 128, 32-byte rows)
    for (uint32_t D = 128; D <= 4096; D *= 2) {
        const size_t b = size_t(INST) * D * WRITERS * seg_cap(D) * 32;
        bytes = b > bytes ? b : bytes;
    }
    bytes += 64u << 20;
    CHECK(hipMalloc(&c.buf, bytes));
    CHECK(hipMalloc(&c.cnt, 64));
    CHECK(hipMemset(c.buf, 0, bytes));
    c.seed = 1;
    const bool all = !std::strcmp(only, "all");
    if (all || !std::strcmp(only, "wr")) {
        // the shipping pattern (4096 buckets, one row per store) and coarser destinations
        run_wr<4096, 1, 8>(c);
        run_wr<4096, 1, 6>(c);
        run_wr<1024, 1, 8>(c);
        run_wr<1024, 1, 6>(c);
        run_wr<512, 1, 8>(c);
        run_wr<256, 1, 8>(c);
        run_wr<256, 1, 6>(c);
        run_wr<128, 1, 8>(c);
        // LDS run buffers
        run_wr<1024, 2, 8>(c);
        run_wr<1024, 2, 6>(c);
        run_wr<512, 2, 8>(c);
        run_wr<512, 4, 8>(c);
        run_wr<512, 4, 6>(c);
        run_wr<256, 4, 8>(c);
        run_wr<256, 4, 6>(c);
        run_wr<256, 8, 6>(c);
        run_wr<256, 8, 4>(c);
        run_wr<128, 8, 8>(c);
    }
    if (all || !std::strcmp(only, "rd")) {
        run_wr<1024, 1, 8>(c);  // fill the layout the reads walk
        run_rd<1024, 8>(c, 1);
        run_rd<1024, 8>(c, 2);
        run_wr<512, 1, 8>(c);
        run_rd<512, 8>(c, 1);
        run_rd<512, 8>(c, 2);
        run_rd<512, 8>(c, 4);
        run_wr<256, 1, 6>(c);
        run_rd<256, 6>(c, 1);
        run_rd<256, 6>(c, 4);
        run_rd<256, 6>(c, 8);
    }
    CHECK(hipFree(c.buf));
    CHECK(hipFree(c.cnt));
    return 0;
}
