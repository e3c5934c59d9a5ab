#!/bin/bash
# Compile the reference's sph sources + tools/ref_x16r_vectors.cpp in /tmp and write
# tests/data/x16r_vectors.json (golden digests for csrc/pow/x16r*.cpp).
set -euo pipefail
REF=${REF:-/root/reference/src}
OUT=${OUT:-/tmp/ref_x16r}
HERE=$(cd "$(dirname "$0")" && pwd)
mkdir -p "$OUT"
for f in blake bmw cubehash echo fugue groestl hamsi jh keccak luffa shabal shavite simd skein whirlpool sph_sha2big; do
  gcc -O2 -w -I"$REF" -c "$REF/algo/$f.c" -o "$OUT/$f.o"
done
g++ -O2 -w -I"$REF" -c "$REF/algo/tiger.cpp" -o "$OUT/tiger.o"
g++ -O2 -std=c++17 -I"$REF" "$HERE/ref_x16r_vectors.cpp" "$OUT"/*.o -o "$OUT/ref_x16r_vectors"
"$OUT/ref_x16r_vectors" > "${1:-$HERE/../tests/data/x16r_vectors.json}"
