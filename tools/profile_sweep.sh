#!/bin/bash
# rocprofv3 of bench.py's own K/M sweep and config-3 windows (bench.py --sweep-only):
# pass 1 kernel trace (durations), passes 2 / 3 kernel trace + one PMC counter each
# (FETCH_SIZE, WRITE_SIZE: separate passes, TCC slots).  Each pass writes the bench's
# JSON for that process, so tools/sweep_trace_summary.py compares every leg's HIP-
# event rate with the rocprof average of the very dispatches it timed.
# Usage: tools/profile_sweep.sh <tag>
set -euo pipefail
TAG=$1
OUT=gpurun_out/sweep_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py --sweep-only --json-out "$OUT/trace.json" > "$OUT/trace.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o run -- python3 bench.py --sweep-only --json-out "$OUT/fetch.json" > "$OUT/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d "$OUT/write" -o run -- python3 bench.py --sweep-only --json-out "$OUT/write.json" > "$OUT/write.log" 2>&1
echo "done $TAG"
