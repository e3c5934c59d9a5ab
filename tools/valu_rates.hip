// Issue rate of the VALU instructions the KawPow round is made of, on one MI355X (gfx950).
//
// Each thread runs 8 independent chains of one instruction (inline asm, so the compiler can
// neither fuse nor drop it) for ITER iterations; 8 waves per SIMD keep the issue port busy. The
// printed cycles assume the 2.4 GHz maximum clock (s_memtime does not tick with the shader clock);
// the exact figure is taken under counters: SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs)
// = wave64 VALU instructions issued per CU per cycle (profiles/r6t_valu_issue: 0.89-0.90 for
// most ops, 1.17 for v_add / v_xor).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/valu_rates tools/valu_rates.hip
//   rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- tools/bin/valu_rates
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

constexpr int ITER = 4096;
constexpr int BLOCK = 512;  // 8 waves: 2 per SIMD per workgroup

#define OP2(name, ins)                                                                      \
    struct name {                                                                           \
        static constexpr const char* tag = ins;                                             \
        __device__ static void run(uint32_t& a, uint32_t b) { asm volatile(ins " %0, %0, %1" : "+v"(a) : "v"(b)); } \
    };
#define OP3(name, ins)                                                                      \
    struct name {                                                                           \
        static constexpr const char* tag = ins;                                             \
        __device__ static void run(uint32_t& a, uint32_t b) {                               \
            asm volatile(ins " %0, %0, %1, %0" : "+v"(a) : "v"(b));                         \
        }                                                                                   \
    };

OP2(Add, "v_add_u32")
OP2(Xor, "v_xor_b32")
OP2(MulLo, "v_mul_lo_u32")
OP2(MulHi, "v_mul_hi_u32")
OP2(Mul24, "v_mul_u32_u24")
OP2(MulHi24, "v_mul_hi_u32_u24")
OP2(Min, "v_min_u32")
OP3(Alignbit, "v_alignbit_b32")
OP3(LshlAdd, "v_lshl_add_u32")
OP3(Xad, "v_xad_u32")
OP3(Mad24, "v_mad_u32_u24")
OP2(And, "v_and_b32")
OP2(Or, "v_or_b32")
OP2(Sub, "v_sub_u32")
OP2(Lshl, "v_lshlrev_b32")
OP2(Lshr, "v_lshrrev_b32")
OP2(Max, "v_max_u32")
OP3(Add3, "v_add3_u32")
OP3(Or3, "v_or3_b32")
OP3(LshlOr, "v_lshl_or_b32")
OP3(AndOr, "v_and_or_b32")
OP3(Perm, "v_perm_b32")
OP3(Bfi, "v_bfi_b32")
OP2(AddE64, "v_add_u32_e64")
OP2(XorE64, "v_xor_b32_e64")
OP2(AndE64, "v_and_b32_e64")
OP2(SubE64, "v_sub_u32_e64")
OP2(MinE64, "v_min_u32_e64")
OP2(Mul24E64, "v_mul_u32_u24_e64")
OP2(LshlE64, "v_lshlrev_b32_e64")
struct Bitop3b {
    static constexpr const char* tag = "v_bitop3_b32 (0x6c)";
    __device__ static void run(uint32_t& a, uint32_t b) { asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x6c" : "+v"(a) : "v"(b)); }
};
struct AlignbitImm {
    static constexpr const char* tag = "v_alignbit_b32 (rotate by an inline constant)";
    __device__ static void run(uint32_t& a, uint32_t) { asm volatile("v_alignbit_b32 %0, %0, %0, 13" : "+v"(a)); }
};
struct AddSgpr {
    static constexpr const char* tag = "v_add_u32 (SGPR operand)";
    __device__ static void run(uint32_t& a, uint32_t b) { asm volatile("v_add_u32 %0, %1, %0" : "+v"(a) : "s"(b)); }
};

struct Bitop3 {
    static constexpr const char* tag = "v_bitop3_b32 (0x96: 3-way xor)";
    __device__ static void run(uint32_t& a, uint32_t b) { asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a) : "v"(b)); }
};
struct Bcnt {
    static constexpr const char* tag = "v_bcnt_u32_b32";
    __device__ static void run(uint32_t& a, uint32_t b) { asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(a) : "v"(b)); }
};
struct Ffbh {
    static constexpr const char* tag = "v_ffbh_u32";
    __device__ static void run(uint32_t& a, uint32_t) { asm volatile("v_ffbh_u32 %0, %0" : "+v"(a)); }
};
struct MovDpp {
    static constexpr const char* tag = "v_mov_b32_dpp row_newbcast:1";
    __device__ static void run(uint32_t& a, uint32_t) {
        asm volatile("s_nop 1\n v_mov_b32_dpp %0, %0 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(a));
    }
};

struct MadU64 {
    static constexpr const char* tag = "v_mad_u64_u32";
    __device__ static void run(uint32_t& a, uint32_t b) {
        uint64_t r;
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b) : "vcc");
        a = (uint32_t)r ^ (uint32_t)(r >> 32);
    }
};

template <class Op>
__global__ __launch_bounds__(BLOCK) void bench(uint32_t* out, uint64_t* cycles, uint32_t seed) {
    uint32_t a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = seed + threadIdx.x * 8 + k;
    const uint32_t b = seed | 1u;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < ITER; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) Op::run(a[k], b);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) x ^= a[k];
    out[blockIdx.x * BLOCK + threadIdx.x] = x;
    if (threadIdx.x == 0) cycles[blockIdx.x] = t1 - t0;
}

template <class Op>
static void run(uint32_t* out, uint64_t* cyc, int blocks) {
    bench<Op><<<blocks, BLOCK>>>(out, cyc, 7);  // warm
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    bench<Op><<<blocks, BLOCK>>>(out, cyc, 9);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    // wave64 instructions issued per SIMD: blocks x 8 waves x ITER x 8 over (CUs x 4 SIMDs)
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    int khz = 0;
    CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, 0));
    const double per_simd = double(blocks) * (BLOCK / 64) * ITER * 8 / (double(cus) * 4);
    const double cycles_at_max = ms * 1e-3 * khz * 1e3;
    // the shader-clock cycles one workgroup measured itself (s_memtime): its 2 waves per SIMD
    // interleave with the 6 of the other 3 workgroups on that SIMD, so SIMD cycles per wave op =
    // elapsed / (8 waves x ITER x 8 ops)
    uint64_t c0 = 0;
    CHECK(hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost));
    const double sclk_cycles = double(c0) / (8.0 * ITER * 8);
    std::printf("{\"op\":\"%s\",\"ms\":%.3f,\"cycles_per_wave_op_at_max_clock\":%.2f,"
                "\"cycles_per_wave_op_memtime\":%.2f,\"implied_mhz\":%.0f}\n", Op::tag, ms,
                cycles_at_max / per_simd, sclk_cycles, double(c0) / (ms * 1e3));
    std::fflush(stdout);
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = cus * 4;  // 4 workgroups of 8 waves per CU: 8 waves per SIMD
    uint32_t* out = nullptr;
    uint64_t* cyc = nullptr;
    CHECK(hipMalloc(&out, size_t(blocks) * BLOCK * 4));
    CHECK(hipMalloc(&cyc, size_t(blocks) * 8));
    run<Add>(out, cyc, blocks);
    run<Xor>(out, cyc, blocks);
    run<Min>(out, cyc, blocks);
    run<Alignbit>(out, cyc, blocks);
    run<LshlAdd>(out, cyc, blocks);
    run<Xad>(out, cyc, blocks);
    run<Mul24>(out, cyc, blocks);
    run<Mad24>(out, cyc, blocks);
    run<MulHi24>(out, cyc, blocks);
    run<MulLo>(out, cyc, blocks);
    run<MulHi>(out, cyc, blocks);
    run<MadU64>(out, cyc, blocks);
    run<And>(out, cyc, blocks);
    run<Or>(out, cyc, blocks);
    run<Sub>(out, cyc, blocks);
    run<Lshl>(out, cyc, blocks);
    run<Lshr>(out, cyc, blocks);
    run<Max>(out, cyc, blocks);
    run<Add3>(out, cyc, blocks);
    run<Or3>(out, cyc, blocks);
    run<LshlOr>(out, cyc, blocks);
    run<AndOr>(out, cyc, blocks);
    run<Perm>(out, cyc, blocks);
    run<Bfi>(out, cyc, blocks);
    run<AddE64>(out, cyc, blocks);
    run<XorE64>(out, cyc, blocks);
    run<AndE64>(out, cyc, blocks);
    run<SubE64>(out, cyc, blocks);
    run<MinE64>(out, cyc, blocks);
    run<Mul24E64>(out, cyc, blocks);
    run<LshlE64>(out, cyc, blocks);
    run<Bitop3b>(out, cyc, blocks);
    run<AlignbitImm>(out, cyc, blocks);
    run<AddSgpr>(out, cyc, blocks);
    run<Add>(out, cyc, blocks);
    run<Bitop3>(out, cyc, blocks);
    run<Bcnt>(out, cyc, blocks);
    run<Ffbh>(out, cyc, blocks);
    run<MovDpp>(out, cyc, blocks);
    CHECK(hipFree(out));
    CHECK(hipFree(cyc));
    return 0;
}
