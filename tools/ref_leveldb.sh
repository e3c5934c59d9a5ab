#!/bin/bash
# Build the reference's LevelDB (src/leveldb, compiled from source, POSIX port, no snappy) and
# tools/ref_leveldb_tool.cpp into $OUT (default build/ref_leveldb/, git-ignored). Prints the
# tool's path. Used by tests/test_ldb.py to cross-check the on-disk format both ways.
set -euo pipefail
REF=${REF:-/root/reference/src/leveldb}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=${OUT:-$HERE/../build/ref_leveldb}
mkdir -p "$OUT/obj"
TOOL="$OUT/ref_leveldb_tool"
if [ -x "$TOOL" ] && [ "$TOOL" -nt "$HERE/ref_leveldb_tool.cpp" ]; then echo "$TOOL"; exit 0; fi
FLAGS="-O2 -std=c++11 -w -DLEVELDB_PLATFORM_POSIX -DOS_LINUX -DLEVELDB_ATOMIC_PRESENT -I$REF -I$REF/include"
SRCS=$(ls "$REF"/db/*.cc "$REF"/table/*.cc "$REF"/util/*.cc "$REF"/port/port_posix.cc "$REF"/port/port_posix_sse.cc \
  | grep -v -E '_test\.cc$|_bench\.cc$|db_bench|leveldbutil|testharness|testutil|env_win|/c\.cc$')
pids=()
for s in $SRCS; do
  o="$OUT/obj/$(basename "$(dirname "$s")")_$(basename "$s" .cc).o"
  extra=""
  case "$s" in *port_posix_sse.cc) extra="-msse4.2";; esac
  g++ $FLAGS $extra -c "$s" -o "$o" &
  pids+=($!)
  if [ ${#pids[@]} -ge 8 ]; then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
done
for p in "${pids[@]}"; do wait "$p"; done
g++ $FLAGS "$HERE/ref_leveldb_tool.cpp" "$OUT"/obj/*.o -lpthread -o "$TOOL"
echo "$TOOL"
