#!/bin/bash
# Compile the reference's HAVAL / Lyra2 sources + tools/ref_legacy_vectors.cpp in /tmp and write
# tests/data/legacy_algo_vectors.json (golden digests for csrc/pow/legacy_algos.cpp).
set -euo pipefail
REF=${REF:-/root/reference/src}
OUT=${OUT:-/tmp/ref_legacy}
HERE=$(cd "$(dirname "$0")" && pwd)
mkdir -p "$OUT"
gcc -O2 -w -I"$REF" -c "$REF/algo/haval.c" -o "$OUT/haval.o"
g++ -O2 -w -I"$REF" -c "$REF/algo/lyra2.cpp" -o "$OUT/lyra2.o"
g++ -O2 -w -I"$REF" -c "$REF/algo/sponge.cpp" -o "$OUT/sponge.o"
g++ -O2 -std=c++17 -I"$REF" "$HERE/ref_legacy_vectors.cpp" "$OUT"/*.o -o "$OUT/ref_legacy_vectors"
"$OUT/ref_legacy_vectors" > "${1:-$HERE/../tests/data/legacy_algo_vectors.json}"
