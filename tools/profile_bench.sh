#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box via gpurun).
#   pass 1: kernel trace + stats (durations)
#   pass 2: FETCH_SIZE only      pass 3: WRITE_SIZE only  (separate --pmc passes;
#   TCC slots: FETCH_SIZE costs 3, WRITE_SIZE 2 -> cannot share a pass on gfx950)
# Usage: tools/profile_bench.sh <tag> [extra bench args...]
set -euo pipefail
TAG=${1:-r01}; shift || true
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 3 --no-extras --no-cpu $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
find "$OUT" -name '*.csv' | head -50
