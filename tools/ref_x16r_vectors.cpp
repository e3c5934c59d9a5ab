// Golden-vector harness for the X16R / X16RV2 primitives.
//
// Linked against the reference's own sph sources (compiled in /tmp by
// tools/ref_x16r_vectors.sh; nothing from them is copied into this repo). Emits
// JSON: per-primitive digests over deterministic inputs of several lengths, and
// whole X16R / X16RV2 hashes of synthetic 80-byte headers under several
// hashPrevBlock values (chaining per src/hash.h:335-605, selection per
// src/hash.h:320-327). tests/test_x16r.py checks csrc/pow/x16r*.cpp against it.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
#include "algo/sph_blake.h"
#include "algo/sph_bmw.h"
#include "algo/sph_cubehash.h"
#include "algo/sph_echo.h"
#include "algo/sph_fugue.h"
#include "algo/sph_groestl.h"
#include "algo/sph_hamsi.h"
#include "algo/sph_jh.h"
#include "algo/sph_keccak.h"
#include "algo/sph_luffa.h"
#include "algo/sph_sha2.h"
#include "algo/sph_shabal.h"
#include "algo/sph_shavite.h"
#include "algo/sph_simd.h"
#include "algo/sph_skein.h"
#include "algo/sph_whirlpool.h"
}
#include "algo/sph_tiger.h"

typedef void (*init_fn)(void*);
typedef void (*upd_fn)(void*, const void*, size_t);
typedef void (*close_fn)(void*, void*);

struct Algo { const char* name; init_fn i; upd_fn u; close_fn c; int out; };

static const Algo kAlgos[17] = {
    {"blake512", sph_blake512_init, sph_blake512, sph_blake512_close, 64},
    {"bmw512", sph_bmw512_init, sph_bmw512, sph_bmw512_close, 64},
    {"groestl512", sph_groestl512_init, sph_groestl512, sph_groestl512_close, 64},
    {"jh512", sph_jh512_init, sph_jh512, sph_jh512_close, 64},
    {"keccak512", sph_keccak512_init, sph_keccak512, sph_keccak512_close, 64},
    {"skein512", sph_skein512_init, sph_skein512, sph_skein512_close, 64},
    {"luffa512", sph_luffa512_init, sph_luffa512, sph_luffa512_close, 64},
    {"cubehash512", sph_cubehash512_init, sph_cubehash512, sph_cubehash512_close, 64},
    {"shavite512", sph_shavite512_init, sph_shavite512, sph_shavite512_close, 64},
    {"simd512", sph_simd512_init, sph_simd512, sph_simd512_close, 64},
    {"echo512", sph_echo512_init, sph_echo512, sph_echo512_close, 64},
    {"hamsi512", sph_hamsi512_init, sph_hamsi512, sph_hamsi512_close, 64},
    {"fugue512", sph_fugue512_init, sph_fugue512, sph_fugue512_close, 64},
    {"shabal512", sph_shabal512_init, sph_shabal512, sph_shabal512_close, 64},
    {"whirlpool", sph_whirlpool_init, sph_whirlpool, sph_whirlpool_close, 64},
    {"sha512", sph_sha512_init, sph_sha512, sph_sha512_close, 64},
    {"tiger", sph_tiger_init, sph_tiger, sph_tiger_close, 24},
};

static unsigned char g_ctx[1 << 16];

static void run(int a, const unsigned char* in, size_t n, unsigned char out[64]) {
    std::memset(out, 0, 64);
    kAlgos[a].i(g_ctx);
    kAlgos[a].u(g_ctx, in, n);
    kAlgos[a].c(g_ctx, out);
}

static std::string hex(const unsigned char* p, size_t n) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < n; ++i) { s += d[p[i] >> 4]; s += d[p[i] & 15]; }
    return s;
}

static uint64_t g_rng = 0x9E3779B97F4A7C15ULL;
static unsigned char rnd() {
    g_rng ^= g_rng << 13; g_rng ^= g_rng >> 7; g_rng ^= g_rng << 17;
    return (unsigned char)(g_rng >> 32);
}

static int selection(const unsigned char prev[32], int i) {
    const int k = 63 - (48 + i);
    return (k & 1) ? (prev[k / 2] >> 4) : (prev[k / 2] & 15);
}

static void x16r(const unsigned char* in, size_t n, const unsigned char prev[32], bool v2, unsigned char out[32]) {
    unsigned char h[64], t[64];
    const unsigned char* p = in;
    size_t len = n;
    for (int i = 0; i < 16; ++i) {
        const int s = selection(prev, i);
        if (v2 && (s == 4 || s == 6 || s == 15)) {
            run(16, p, len, t);  // tiger-192, zero-extended to 64 bytes
            run(s, t, 64, h);
        } else {
            unsigned char tmp[64];
            run(s, p, len, tmp);
            std::memcpy(h, tmp, 64);
        }
        p = h;
        len = 64;
    }
    std::memcpy(out, h, 32);
}

int main() {
    const size_t lens[] = {0, 1, 3, 31, 32, 55, 63, 64, 65, 80, 111, 112, 127, 128, 129, 191, 255, 256, 300, 1000};
    std::printf("{\n \"primitives\": {\n");
    for (int a = 0; a < 17; ++a) {
        std::printf("  \"%s\": [", kAlgos[a].name);
        g_rng = 0x9E3779B97F4A7C15ULL + a;
        bool first = true;
        for (size_t n : lens) {
            std::vector<unsigned char> in(n);
            for (auto& c : in) c = rnd();
            unsigned char out[64];
            run(a, in.data(), n, out);
            std::printf("%s\n   [\"%s\", \"%s\"]", first ? "" : ",", hex(in.data(), n).c_str(),
                        hex(out, kAlgos[a].out).c_str());
            first = false;
        }
        std::printf("\n  ]%s\n", a == 16 ? "" : ",");
    }
    std::printf(" },\n \"chains\": [");
    g_rng = 0xC0FFEEULL;
    for (int k = 0; k < 48; ++k) {
        unsigned char hdr[80], prev[32], o1[32], o2[32];
        for (auto& c : hdr) c = rnd();
        for (auto& c : prev) c = rnd();
        if (k < 16) {  // force every algorithm into slot 0..15 at least once
            for (int i = 0; i < 16; ++i) {
                const int kk = 63 - (48 + i), s = (k + i) & 15;
                prev[kk / 2] = (kk & 1) ? (unsigned char)((prev[kk / 2] & 0x0F) | (s << 4))
                                        : (unsigned char)((prev[kk / 2] & 0xF0) | s);
            }
        }
        std::memcpy(hdr + 4, prev, 32);
        x16r(hdr, 80, prev, false, o1);
        x16r(hdr, 80, prev, true, o2);
        std::printf("%s\n  {\"header\": \"%s\", \"prev\": \"%s\", \"x16r\": \"%s\", \"x16rv2\": \"%s\"}", k ? "," : "",
                    hex(hdr, 80).c_str(), hex(prev, 32).c_str(), hex(o1, 32).c_str(), hex(o2, 32).c_str());
    }
    std::printf("\n ]\n}\n");
    return 0;
}
