#!/bin/bash
# Compute-free ceilings of every K/M-sweep and config-3 leg on the shipped launch
# shapes: bench.py --sweep-only runs twice on the same box, once
# with the shipped librsgpu.so and once with its RS_PATTERN_ONLY=1 twin
# (abx/pattern.so, built on the CPU by tools/build_ab.sh pattern ... -DRS_PATTERN_ONLY=1):
# the same kernels, launches, tasks, loads and stores with the GF(2^8) arithmetic
# replaced by one XOR per input dword, timed at several occupancy caps.
# The twin is loaded by path (RSGPU_LIB, _lib.py): the shipped library is never
# overwritten, so a run killed half way leaves nothing wrong behind.
# tools/ceiling_summary.py pairs the legs.
# Usage: tools/ceiling_probe.sh <tag>
set -euo pipefail
TAG=$1
OUT=gpurun_out/ceiling_${TAG}
TWIN=$(pwd)/abx/pattern.so
mkdir -p "$OUT"
test -f "$TWIN"
timeout -k 10 400 python3 bench.py --sweep-only --json-out "$OUT/shipped.json" > "$OUT/shipped.log" 2>&1
# the twin at several occupancies (rs_set_occupancy_cap; 0 = uncapped): it needs far
# fewer registers than the kernel it mirrors, so left alone it runs more waves per
# SIMD, which these streaming patterns do not always want -- the ceiling is the best
# the pattern reaches at any of them
for C in ${CAPS:-0 2 3 4 6}; do
  RSGPU_LIB=$TWIN timeout -k 10 400 python3 bench.py --sweep-only --occ-cap $C \
    --json-out "$OUT/pattern_c$C.json" > "$OUT/pattern_c$C.log" 2>&1
done
python3 tools/ceiling_summary.py "$OUT" "$TAG"
