#!/bin/bash
# Build the reference's ethash/ProgPoW sources + tools/ref_cpu_baseline.cpp in /tmp and run it.
# Output: one JSON line (MH/s of progpow::search on all host cores). Used for BASELINE.md.
set -euo pipefail
REF=${REF:-/root/reference/src}
OUT=${OUT:-/tmp/ref_cpu_baseline}
HERE=$(cd "$(dirname "$0")" && pwd)
mkdir -p "$OUT"
E=$REF/crypto/ethash/lib
for f in keccak/keccak.c keccak/keccakf1600.c keccak/keccakf800.c ethash/primes.c; do
  gcc -O3 -march=native -I"$REF" -c "$E/$f" -o "$OUT/$(basename "$f").o"
done
for f in ethash/ethash.cpp ethash/progpow.cpp; do
  g++ -std=c++17 -O3 -march=native -I"$REF" -c "$E/$f" -o "$OUT/$(basename "$f").o"
done
g++ -std=c++17 -O3 -march=native -I"$REF" "$HERE/ref_cpu_baseline.cpp" "$OUT"/*.o -lpthread -o "$OUT/ref_cpu_baseline"
"$OUT/ref_cpu_baseline" "${1:-384}" "${2:-20}"
