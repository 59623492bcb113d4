#!/bin/bash
# HBM traffic (rocprofv3 PMC, separate FETCH_SIZE / WRITE_SIZE passes) and kernel
# durations for single workloads of tools/ab_bench.py, one process per workload so
# each kernel's dispatches belong to one shape.  The trace pass times >= 100 ms of
# back-to-back launches (MIN_MS), the window bench.py's K/M sweep times, so the
# averages describe the same sustained clock.
# Usage: [AB_EXTRA=--parity-pad] tools/profile_kmsweep_pmc.sh <tag> <workload>...
set -euo pipefail
TAG=$1; shift
export TMPDIR=/tmp
for W in "$@"; do
  OUT=gpurun_out/pmc_${TAG}/$W
  mkdir -p "$OUT"
  ARGS="--rounds 1 --iters 6 --bpc 0 --workloads $W ${AB_EXTRA:-}"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 tools/ab_bench.py $ARGS --min-ms ${MIN_MS:-100} > "$OUT/trace.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o run -- python3 tools/ab_bench.py $ARGS > "$OUT/fetch.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/write" -o run -- python3 tools/ab_bench.py $ARGS > "$OUT/write.log" 2>&1
  echo "done $W"
done
