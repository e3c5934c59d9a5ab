// Golden-vector harness for csrc/pow/legacy_algos.cpp: links the reference's own HAVAL and Lyra2
// sources (compiled in /tmp by tools/ref_legacy_vectors.sh, never shipped) and prints JSON.
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

extern "C" {
#include "algo/sph_haval.h"
}
#include "algo/lyra2.h"

static std::string hex(const unsigned char* p, size_t n) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < n; ++i) { s += d[p[i] >> 4]; s += d[p[i] & 15]; }
    return s;
}

static std::vector<unsigned char> msg(size_t n, unsigned seed) {
    std::vector<unsigned char> m(n);
    uint32_t x = 0x9e3779b9u * (seed + 1);
    for (size_t i = 0; i < n; ++i) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; m[i] = (unsigned char)x; }
    return m;
}

typedef void (*init_f)(void*);
typedef void (*upd_f)(void*, const void*, size_t);
typedef void (*close_f)(void*, void*);

#define HV(bits, p) {bits, p, sph_haval##bits##_##p##_init, sph_haval##bits##_##p, sph_haval##bits##_##p##_close}
struct Hv { int bits, passes; init_f i; upd_f u; close_f c; };

int main() {
    const Hv hv[] = {HV(128, 3), HV(128, 4), HV(128, 5), HV(160, 3), HV(160, 4), HV(160, 5), HV(192, 3), HV(192, 4),
                     HV(192, 5), HV(224, 3), HV(224, 4), HV(224, 5), HV(256, 3), HV(256, 4), HV(256, 5)};
    const size_t lens[] = {0, 1, 3, 80, 117, 118, 119, 127, 128, 129, 255, 300};
    std::printf("{\"haval\": [\n");
    bool first = true;
    for (const Hv& h : hv)
        for (size_t li = 0; li < sizeof lens / sizeof lens[0]; ++li) {
            std::vector<unsigned char> m = msg(lens[li], unsigned(li));
            sph_haval_context cc;
            unsigned char out[32];
            h.i(&cc);
            h.u(&cc, m.data(), m.size());
            h.c(&cc, out);
            std::printf("%s {\"passes\": %d, \"bits\": %d, \"msg\": \"%s\", \"digest\": \"%s\"}", first ? "" : ",\n",
                        h.passes, h.bits, hex(m.data(), m.size()).c_str(), hex(out, size_t(h.bits / 8)).c_str());
            first = false;
        }
    std::printf("\n], \"lyra2\": [\n");
    struct L { size_t pwd, salt; uint64_t klen, t, rows, cols; int old; };
    const L ls[] = {{32, 32, 32, 1, 4, 4, 0}, {32, 32, 32, 1, 8, 8, 1}, {32, 32, 32, 1, 8, 8, 0}, {32, 32, 64, 2, 4, 4, 0},
                    {10, 6, 100, 3, 16, 2, 0}, {80, 80, 200, 1, 4, 4, 0}, {80, 80, 32, 2, 8, 3, 1}, {5, 0, 32, 4, 32, 1, 0},
                    {32, 32, 96, 1, 4, 1, 0}, {32, 32, 97, 2, 4, 2, 1}};
    first = true;
    for (size_t i = 0; i < sizeof ls / sizeof ls[0]; ++i) {
        const L& l = ls[i];
        std::vector<unsigned char> pwd = msg(l.pwd, 100 + unsigned(i)), salt = msg(l.salt, 200 + unsigned(i));
        std::vector<unsigned char> k(l.klen);
        int rc = l.old ? LYRA2_old(k.data(), l.klen, pwd.data(), l.pwd, salt.data(), l.salt, l.t, l.rows, l.cols)
                       : LYRA2(k.data(), l.klen, pwd.data(), l.pwd, salt.data(), l.salt, l.t, l.rows, l.cols);
        std::printf("%s {\"pwd\": \"%s\", \"salt\": \"%s\", \"klen\": %llu, \"time_cost\": %llu, \"n_rows\": %llu, "
                    "\"n_cols\": %llu, \"old\": %s, \"rc\": %d, \"key\": \"%s\"}",
                    first ? "" : ",\n", hex(pwd.data(), pwd.size()).c_str(), hex(salt.data(), salt.size()).c_str(),
                    (unsigned long long)l.klen, (unsigned long long)l.t, (unsigned long long)l.rows,
                    (unsigned long long)l.cols, l.old ? "true" : "false", rc, hex(k.data(), k.size()).c_str());
        first = false;
    }
    std::printf("\n]}\n");
    return 0;
}
