// Probe variants of kawpow_verify_waves (hip/kernels/kawpow_verify_light.hip) for
// tools/verify_waves_probe.py: where a round's ~7 us goes. Not product code.
//
//   V0  the shipping kernel's round (sanity: same time as kawpow_verify_waves)
//   V1  no L1 lookups (the cache ops merge the source register itself)     timing only
//   V2  fixed op kinds (math xor, merge rotl-xor): no scalar branch trees   timing only
//   V3  no DAG load (the merge words are the index)                          timing only
//   V4  fixed registers (op i reads/writes i % 32): no gpr_idx moves         timing only
//   V5  branch-free merges (masks from the op word on the SALU), bit-exact
//   V6  jump-table dispatch (s_getpc / s_setpc into fixed-size handler slots) for math and merges
//   V7  jump-table merges, branch-tree math
//   V8  jump-table math, branch-tree merges
//   V9  one shared handler table called per op (math + merge fused): kwt_* of the shipping kernel
//   V10 V9 + a cache op fused into the math op after it when their registers do not overlap
#include "kawpow_verify_light.hip"

// kind-indexed handler slots inside one asm block: s_getpc gives the address after itself, the
// slot offset is 24 bytes (the 5 dispatch instructions + s_setpc) + kind * slot size; `.org`
// fixes every slot's start (and refuses a handler that outgrows its slot at assembly time)
NX_DEV uint32_t pj_math(uint32_t a, uint32_t b, uint32_t kind) {
    uint32_t d, t;
    asm volatile(
        "s_getpc_b64 s[98:99]\n"
        "s_min_u32 s97, %[k], 10\n"
        "s_lshl_b32 s97, s97, 5\n"
        "s_add_u32 s97, s97, 24\n"
        "s_add_u32 s98, s98, s97\n"
        "s_addc_u32 s99, s99, 0\n"
        "s_setpc_b64 s[98:99]\n"
        ".Lkb%=:\n"
        "v_add_u32_e32 %[d], %[a], %[b]\n s_branch .Lke%=\n"
        ".org .Lkb%=+32\n"
        "v_mul_lo_u32 %[d], %[a], %[b]\n s_branch .Lke%=\n"
        ".org .Lkb%=+64\n"
        "v_mul_hi_u32 %[d], %[a], %[b]\n s_branch .Lke%=\n"
        ".org .Lkb%=+96\n"
        "v_min_u32_e32 %[d], %[a], %[b]\n s_branch .Lke%=\n"
        ".org .Lkb%=+128\n"
        "v_sub_u32_e32 %[t], 0, %[b]\n v_alignbit_b32 %[d], %[a], %[a], %[t]\n s_branch .Lke%=\n"
        ".org .Lkb%=+160\n"
        "v_alignbit_b32 %[d], %[a], %[a], %[b]\n s_branch .Lke%=\n"
        ".org .Lkb%=+192\n"
        "v_and_b32_e32 %[d], %[a], %[b]\n s_branch .Lke%=\n"
        ".org .Lkb%=+224\n"
        "v_or_b32_e32 %[d], %[a], %[b]\n s_branch .Lke%=\n"
        ".org .Lkb%=+256\n"
        "v_xor_b32_e32 %[d], %[a], %[b]\n s_branch .Lke%=\n"
        ".org .Lkb%=+288\n"
        "v_ffbh_u32_e32 %[t], %[a]\n v_min_u32_e32 %[t], 32, %[t]\n v_ffbh_u32_e32 %[d], %[b]\n"
        " v_min_u32_e32 %[d], 32, %[d]\n v_add_u32_e32 %[d], %[t], %[d]\n s_branch .Lke%=\n"
        ".org .Lkb%=+320\n"
        "v_bcnt_u32_b32 %[t], %[a], 0\n v_bcnt_u32_b32 %[d], %[b], %[t]\n"
        ".Lke%=:\n"
        : [d] "=&v"(d), [t] "=&v"(t)
        : [a] "v"(a), [b] "v"(b), [k] "s"(kind)
        : "s97", "s98", "s99", "scc");
    return d;
}

NX_DEV uint32_t pj_merge(uint32_t a, uint32_t b, uint32_t kind, uint32_t rot) {
    uint32_t d, t;
    asm volatile(
        "s_sub_u32 s96, 0, %[r]\n"
        "s_getpc_b64 s[98:99]\n"
        "s_and_b32 s97, %[k], 3\n"
        "s_lshl_b32 s97, s97, 4\n"
        "s_add_u32 s97, s97, 24\n"
        "s_add_u32 s98, s98, s97\n"
        "s_addc_u32 s99, s99, 0\n"
        "s_setpc_b64 s[98:99]\n"
        ".Lmb%=:\n"
        "v_lshl_add_u32 %[t], %[a], 5, %[a]\n v_add_u32_e32 %[d], %[t], %[b]\n s_branch .Lme%=\n"
        ".org .Lmb%=+16\n"
        "v_xor_b32_e32 %[t], %[a], %[b]\n v_lshl_add_u32 %[d], %[t], 5, %[t]\n s_branch .Lme%=\n"
        ".org .Lmb%=+32\n"
        "v_alignbit_b32 %[t], %[a], %[a], s96\n v_xor_b32_e32 %[d], %[t], %[b]\n s_branch .Lme%=\n"
        ".org .Lmb%=+48\n"
        "v_alignbit_b32 %[t], %[a], %[a], %[r]\n v_xor_b32_e32 %[d], %[t], %[b]\n"
        ".Lme%=:\n"
        : [d] "=&v"(d), [t] "=&v"(t)
        : [a] "v"(a), [b] "v"(b), [k] "s"(kind), [r] "s"(rot)
        : "s96", "s97", "s98", "s99", "scc");
    return d;
}



// ---- V10: V9's table plus 176 fused slots (cache merge gc, math m, merge gm) at 48 + 44 gc + 4 m + gm:
// a cache op and the math op after it in one call when the cache op's destination is none of the
// math op's registers (else the two V9 calls). Extra registers: v59 = the cache destination's
// value in and out, v58 = the L1 word, s93 = the cache merge rotation.
#define KWC0 "v_lshl_add_u32 v59, v59, 5, v59\n v_add_u32_e32 v59, v59, v58\n"
#define KWC1 "v_xor_b32_e32 v59, v59, v58\n v_lshl_add_u32 v59, v59, 5, v59\n"
#define KWC2 "s_sub_u32 s97, 0, s93\n v_alignbit_b32 v59, v59, v59, s97\n v_xor_b32_e32 v59, v59, v58\n"
#define KWC3 "v_alignbit_b32 v59, v59, v59, s93\n v_xor_b32_e32 v59, v59, v58\n"
#define KWF4(c, m, n0) KWS(n0, KWC##c KWM##m KWG0) KWS(n0 + 1, KWC##c KWM##m KWG1) KWS(n0 + 2, KWC##c KWM##m KWG2) \
    KWS(n0 + 3, KWC##c KWM##m KWG3)
#define KWF44(c, n0) KWF4(c, 0, n0) KWF4(c, 1, n0 + 4) KWF4(c, 2, n0 + 8) KWF4(c, 3, n0 + 12) KWF4(c, 4, n0 + 16) \
    KWF4(c, 5, n0 + 20) KWF4(c, 6, n0 + 24) KWF4(c, 7, n0 + 28) KWF4(c, 8, n0 + 32) KWF4(c, 9, n0 + 36) KWF4(c, 10, n0 + 40)

NX_DEV void kwt2_table(uint32_t& lo, uint32_t& hi) {
    asm volatile(
        "s_getpc_b64 s[94:95]\n"
        ".Lkwt_pc%=:\n"
        "s_add_u32 %[lo], s94, .Lkwt_tab%=-.Lkwt_pc%=\n"
        "s_addc_u32 %[hi], s95, 0\n"
        "s_branch .Lkwt_end%=\n"
        ".p2align 6\n"
        ".Lkwt_tab%=:\n"
        KWS4(0, 0) KWS4(1, 4) KWS4(2, 8) KWS4(3, 12) KWS4(4, 16) KWS4(5, 20) KWS4(6, 24) KWS4(7, 28)
        KWS4(8, 32) KWS4(9, 36) KWS4(10, 40)
        KWS(44, KWG0) KWS(45, KWG1) KWS(46, KWG2) KWS(47, KWG3)
        KWF44(0, 48) KWF44(1, 92) KWF44(2, 136) KWF44(3, 180)
        ".org .Lkwt_tab%=+224*64\n"
        ".Lkwt_end%=:\n"
        : [lo] "=s"(lo), [hi] "=s"(hi)
        :
        : "s94", "s95", "scc");
}

// dc = merge_c(dc, lv); d = merge_m(d, math(a, b)) in one call
NX_DEV void kwt_fused(uint32_t lo, uint32_t hi, uint32_t a, uint32_t b, uint32_t& d, uint32_t& dc, uint32_t lv,
                      uint32_t ckind, uint32_t crot, uint32_t kind, uint32_t mkind, uint32_t rot) {
    const uint32_t off = (48u + (ckind & 3u) * 44u + (kind < 10u ? kind : 10u) * 4u + (mkind & 3u)) << 6;
    asm volatile(
        "s_add_u32 s94, %[lo], %[off]\n"
        "s_addc_u32 s95, %[hi], 0\n"
        "s_swappc_b64 s[98:99], s[94:95]\n"
        : "+{v63}"(d), "+{v62}"(b), "+{v59}"(dc)
        : "{v61}"(a), "{v58}"(lv), "{s96}"(rot), "{s93}"(crot), [lo] "s"(lo), [hi] "s"(hi), [off] "s"(off)
        : "v60", "s94", "s95", "s97", "s98", "s99", "scc");
}

template <int V>
NX_DEV uint32_t pv_merge(uint32_t a, uint32_t b, uint32_t kind, uint32_t rot) {
    if constexpr (V == 2) {
        return __builtin_rotateleft32(a, rot) ^ b;
    } else if constexpr (V == 5) {
        // kind 0: a*33 + b, 1: (a^b)*33, 2: rotl(a,r)^b, 3: rotr(a,r)^b -- every select uniform
        const uint32_t m1 = kind == 1 ? ~0u : 0u;
        const uint32_t sr = kind == 2 ? ((32u - rot) & 31u) : (kind == 3 ? (rot & 31u) : 0u);
        const uint32_t mk = kind < 2 ? ~0u : 0u;
        const uint32_t ma = kind == 0 ? ~0u : 0u;
        const uint32_t mx = kind >= 2 ? ~0u : 0u;
        uint32_t t = a ^ (b & m1);
        t = __builtin_amdgcn_alignbit(t, t, sr);
        t = t + ((t & mk) << 5);
        return (t + (b & ma)) ^ (b & mx);
    } else if constexpr (V == 6 || V == 7) {
        return pj_merge(a, b, kind, rot);
    } else {
        return kl_merge(a, b, kind, rot);
    }
}

template <int V>
NX_DEV uint32_t pv_math(uint32_t a, uint32_t b, uint32_t kind) {
    if constexpr (V == 2) return a ^ b;
    else if constexpr (V == 6 || V == 8) return pj_math(a, b, kind);
    else return kl_math(a, b, kind);
}

template <int V>
NX_DEV void pv_waves(const KawpowLightParams& p) {
    __shared__ uint32_t l1[4096];
    for (int i = threadIdx.x; i < 4096; i += KL_BLOCK) l1[i] = p.l1[i];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 15;
    const uint32_t g = (threadIdx.x >> 4) & 3;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (KL_BLOCK / 64) + (threadIdx.x >> 6));
    if (wave * 4 >= p.num_slots) return;
    const int32_t first = __builtin_amdgcn_readfirstlane(p.slots[wave * 4]);
    const int32_t row = p.slots[wave * 4 + g];
    const bool valid = row >= 0;
    const uint32_t jj = (uint32_t)(valid ? row : first);
    uint32_t pi = __builtin_amdgcn_readfirstlane(p.job_program[first]);
    pi = pi < p.num_programs ? pi : 0;
    const uint32_t* prog = p.programs + (size_t)pi * KV_PROG_WORDS;
    uint32_t pw[51];
#pragma unroll
    for (int i = 0; i < 51; ++i) pw[i] = __builtin_amdgcn_readfirstlane(prog[i]);
    const KawpowVerifyJob j = p.jobs[jj];
    uint32_t st2[8];
    {
        uint32_t s[25];
#pragma unroll
        for (int i = 0; i < 8; ++i) s[i] = j.header[i];
        s[8] = (uint32_t)j.nonce;
        s[9] = (uint32_t)(j.nonce >> 32);
        const uint32_t pad[15] = {0x72, 0x41, 0x56, 0x45, 0x4E, 0x43, 0x4F, 0x49, 0x4E, 0x4B, 0x41, 0x57, 0x50, 0x4F, 0x57};
#pragma unroll
        for (int i = 0; i < 15; ++i) s[10 + i] = pad[i];
        keccak_f800(s);
#pragma unroll
        for (int i = 0; i < 8; ++i) st2[i] = s[i];
    }
    kw_mix_t mix;
    {
        const uint32_t z0 = kl_fnv1a(0x811c9dc5u, st2[0]);
        const uint32_t w0 = kl_fnv1a(z0, st2[1]);
        const uint32_t jsr0 = kl_fnv1a(w0, lane);
        uint32_t kz = z0, kw = w0, kj = jsr0, kc = kl_fnv1a(jsr0, lane);
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            kz = 36969u * (kz & 0xffffu) + (kz >> 16);
            kw = 18000u * (kw & 0xffffu) + (kw >> 16);
            kc = 69069u * kc + 1234567u;
            kj ^= (kj << 17);
            kj ^= (kj >> 13);
            kj ^= (kj << 5);
            mix[r] = (((kz << 16) + kw) ^ kc) + kj;
        }
    }
    const uint4* dag = (const uint4*)p.dag;
    uint32_t tlo = 0, thi = 0;
    if constexpr (V == 9) kwt_table(tlo, thi);
    if constexpr (V == 10) kwt2_table(tlo, thi);
#pragma unroll 1
    for (uint32_t r = 0; r < 64; ++r) {
        const uint32_t index = kl_mod(__shfl(mix[0], (int)(r & 15), 16), p.items);
        uint4 d;
        if constexpr (V == 3) d = make_uint4(index, index + 1, index + 2, index + 3);
        else d = dag[(size_t)index * 16 + ((lane ^ r) & 15)];
#pragma unroll
        for (int i = 0; i < 51; ++i) asm volatile("" : "+s"(pw[i]));
        if constexpr (V == 10) {
#pragma unroll
            for (int i = 0; i < 18; ++i) {
                const uint32_t op = pw[11 + i];
                const uint32_t mg = pw[29 + i];
                const uint32_t dst = op >> 24;
                if (i < 11) {
                    const uint32_t opc = pw[i];
                    const uint32_t dc = (opc >> 8) & 31;
                    const uint32_t lv = l1[kw_get(mix, opc) & 4095u];
                    if (dc != (op & 31) && dc != ((op >> 8) & 31) && dc != (dst & 31)) {
                        uint32_t d = kw_get(mix, dst), vc = kw_get(mix, dc);
                        kwt_fused(tlo, thi, kw_get(mix, op), kw_get(mix, op >> 8), d, vc, lv, (opc >> 16) & 3, opc >> 24,
                                  (op >> 16) & 15, mg & 3, mg >> 8);
                        kw_set(mix, dc, vc);
                        kw_set(mix, dst, d);
                        continue;
                    }
                    kw_set(mix, dc, kwt_merge(tlo, thi, kw_get(mix, dc), lv, (opc >> 16) & 3, opc >> 24));
                }
                kw_set(mix, dst, kwt_op(tlo, thi, kw_get(mix, op), kw_get(mix, op >> 8), kw_get(mix, dst), (op >> 16) & 15,
                                        mg & 3, mg >> 8));
            }
            const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t op = pw[47 + i];
                kw_set(mix, op, kwt_merge(tlo, thi, kw_get(mix, op), dw[i], (op >> 8) & 3, op >> 16));
            }
            continue;
        }
        if constexpr (V == 9) {
#pragma unroll
            for (int i = 0; i < 18; ++i) {
                if (i < 11) {
                    const uint32_t op = pw[i];
                    const uint32_t dst = (op >> 8) & 31;
                    kw_set(mix, dst, kwt_merge(tlo, thi, kw_get(mix, dst), l1[kw_get(mix, op) & 4095u], (op >> 16) & 3, op >> 24));
                }
                const uint32_t op = pw[11 + i];
                const uint32_t mg = pw[29 + i];
                const uint32_t dst = op >> 24;
                kw_set(mix, dst, kwt_op(tlo, thi, kw_get(mix, op), kw_get(mix, op >> 8), kw_get(mix, dst), (op >> 16) & 15,
                                        mg & 3, mg >> 8));
            }
            const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t op = pw[47 + i];
                kw_set(mix, op, kwt_merge(tlo, thi, kw_get(mix, op), dw[i], (op >> 8) & 3, op >> 16));
            }
            continue;
        }
#pragma unroll
        for (int i = 0; i < 18; ++i) {
            if (i < 11) {
                const uint32_t op = pw[i];
                const uint32_t src = V == 4 ? (uint32_t)((i * 7 + 3) & 31) : op;
                const uint32_t dst = V == 4 ? (uint32_t)((i * 5 + 1) & 31) : ((op >> 8) & 31);
                const uint32_t a = kw_get(mix, src);
                const uint32_t look = V == 1 ? a : l1[a & 4095u];
                kw_set(mix, dst, pv_merge<V>(kw_get(mix, dst), look, (op >> 16) & 3, op >> 24));
            }
            const uint32_t op = pw[11 + i];
            const uint32_t mg = pw[29 + i];
            const uint32_t s1 = V == 4 ? (uint32_t)((i * 3 + 2) & 31) : op;
            const uint32_t s2 = V == 4 ? (uint32_t)((i * 11 + 5) & 31) : (op >> 8);
            const uint32_t dst = V == 4 ? (uint32_t)((i * 13 + 7) & 31) : (op >> 24);
            const uint32_t v = pv_math<V>(kw_get(mix, s1), kw_get(mix, s2), (op >> 16) & 15);
            kw_set(mix, dst, pv_merge<V>(kw_get(mix, dst), v, mg & 3, mg >> 8));
        }
        const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t op = pw[47 + i];
            const uint32_t dst = V == 4 ? (uint32_t)(i * 8) : op;
            kw_set(mix, dst, pv_merge<V>(kw_get(mix, dst), dw[i], (op >> 8) & 3, op >> 16));
        }
    }
    uint32_t lh = 0x811c9dc5u;
#pragma unroll
    for (int r = 0; r < 32; ++r) lh = kl_fnv1a(lh, mix[r]);
    uint32_t digest[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t a = __shfl(lh, k, 16);
        const uint32_t b = __shfl(lh, k + 8, 16);
        digest[k] = kl_fnv1a(kl_fnv1a(0x811c9dc5u, a), b);
    }
    uint32_t st[25];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = st2[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[8 + i] = digest[i];
    const uint32_t pad[9] = {0x72, 0x41, 0x56, 0x45, 0x4E, 0x43, 0x4F, 0x49, 0x4E};
#pragma unroll
    for (int i = 0; i < 9; ++i) st[16 + i] = pad[i];
    keccak_f800(st);
    if (valid && lane == 0) {
        uint32_t* o = p.out + (size_t)row * 16;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            o[k] = digest[k];
            o[8 + k] = st[k];
        }
    }
}

#define PV(n) extern "C" __global__ __launch_bounds__(KL_BLOCK) void pv_waves_##n(KawpowLightParams p) { pv_waves<n>(p); }
PV(0)
PV(1)
PV(2)
PV(3)
PV(4)
PV(5)
PV(6)
PV(7)
PV(8)
PV(9)
PV(10)
