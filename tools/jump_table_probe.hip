// Standalone check of the s_getpc / s_setpc jump-table dispatch (tools/verify_waves_variants.hip
// pj_math / pj_merge): every math and merge kind on 256 lanes, kind uniform per launch.
#include "../tools/verify_waves_variants.hip"

extern "C" __global__ __launch_bounds__(256) void jt_math(const uint32_t* a, const uint32_t* b, uint32_t* out,
                                                          uint32_t kind) {
    const uint32_t i = threadIdx.x;
    const uint32_t k = __builtin_amdgcn_readfirstlane(kind);
    out[i] = pj_math(a[i], b[i], k);
}

extern "C" __global__ __launch_bounds__(256) void jt_merge(const uint32_t* a, const uint32_t* b, uint32_t* out,
                                                           uint32_t kind, uint32_t rot) {
    const uint32_t i = threadIdx.x;
    out[i] = pj_merge(a[i], b[i], __builtin_amdgcn_readfirstlane(kind), __builtin_amdgcn_readfirstlane(rot));
}
