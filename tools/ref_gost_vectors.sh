#!/bin/bash
# Compile the reference's GOST Streebog source into tools/ref_gost_vectors.c in /tmp and write
# tests/data/gost_vectors.json (golden digests for csrc/pow/legacy_algos.cpp gost_streebog) and
# /tmp/ref_gost/tables.json (input of tools/gost_compact_tables.py).
set -euo pipefail
REF=${REF:-/root/reference/src}
OUT=${OUT:-/tmp/ref_gost}
HERE=$(cd "$(dirname "$0")" && pwd)
mkdir -p "$OUT"
gcc -O2 -w -I"$REF" "$HERE/ref_gost_vectors.c" -o "$OUT/ref_gost_vectors"
"$OUT/ref_gost_vectors" t > "$OUT/tables.json"
"$OUT/ref_gost_vectors" > "${1:-$HERE/../tests/data/gost_vectors.json}"
