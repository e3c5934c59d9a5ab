/* Throwaway harness: the reference's GOST Streebog (src/algo/gost_streebog.c, included as source) ->
 * tests/data/gost_vectors.json (no argument) or its tables as JSON ("t", for
 * tools/gost_compact_tables.py). Build: tools/ref_gost_vectors.sh. */
#include <stdio.h>
#include <string.h>
#include "algo/gost_streebog.c"
int main(int argc, char** argv) {
    if (argc > 1 && argv[1][0] == 't') {  /* tables */
        printf("{\"TG\":[");
        for (int i = 0; i < 8; ++i) { printf("%s[", i ? "," : ""); for (int x = 0; x < 256; ++x) printf("%s\"%016llx\"", x ? "," : "", (unsigned long long)TG[i][x]); printf("]"); }
        printf("],\"C\":[");
        for (int i = 0; i < 12; ++i) { printf("%s\"", i ? "," : ""); for (int b = 0; b < 64; ++b) printf("%02x", C[i][b]); printf("\""); }
        printf("]}\n");
        return 0;
    }
    int lens[] = {0, 1, 2, 3, 31, 32, 33, 55, 63, 64, 65, 80, 100, 120, 127, 128, 129, 191, 192, 200, 255, 256, 300, 1000};
    printf("[");
    for (unsigned k = 0; k < sizeof(lens) / sizeof(lens[0]); ++k) {
        unsigned char msg[1000], h512[64], h256[32];
        for (int j = 0; j < lens[k]; ++j) msg[j] = (unsigned char)(j * 37 + 11 + lens[k]);
        sph_gost512(h512, msg, lens[k]);
        sph_gost256(h256, msg, lens[k]);
        printf("%s{\"msg\":\"", k ? "," : "");
        for (int j = 0; j < lens[k]; ++j) printf("%02x", msg[j]);
        printf("\",\"gost512\":\"");
        for (int j = 0; j < 64; ++j) printf("%02x", h512[j]);
        printf("\",\"gost256\":\"");
        for (int j = 0; j < 32; ++j) printf("%02x", h256[j]);
        printf("\"}");
    }
    printf("]\n");
    return 0;
}
