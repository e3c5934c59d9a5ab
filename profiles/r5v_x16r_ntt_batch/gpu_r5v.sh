#!/bin/bash
# r5v: SIMD-512 NTT butterflies batched 4 / 8 / 16 (tools/x16r_b*.hsaco): slot latency + mixed batch
set -o pipefail
O=gpurun_out/r5v
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 16384 --slots 9 2 > $O/base16k.json 2> $O/err.log &&
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 16384 --slots 9 --hsaco tools/x16r_b4.hsaco > $O/b4_16k.json 2>> $O/err.log &&
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 16384 --slots 9 --hsaco tools/x16r_b8.hsaco > $O/b8_16k.json 2>> $O/err.log &&
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 16384 --slots 9 --hsaco tools/x16r_b16.hsaco > $O/b16_16k.json 2>> $O/err.log &&
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 65536 --slots 9 2 > $O/base65k.json 2>> $O/err.log &&
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 65536 --slots 9 --hsaco tools/x16r_b8.hsaco > $O/b8_65k.json 2>> $O/err.log &&
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 65536 --slots 9 --hsaco tools/x16r_b16.hsaco > $O/b16_65k.json 2>> $O/err.log
echo "exit=$?"
