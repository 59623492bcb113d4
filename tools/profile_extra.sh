#!/bin/bash
# rocprofv3 kernel-trace stats (durations) for the kernels outside bench.py's main
# step: scrub (verify_kernel) and the 64 KiB K/M sweep, at the default occupancy.
# Usage: tools/profile_extra.sh <tag>
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}_extra
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 tools/ab_bench.py \
  --rounds 1 --iters 10 --bpc 0 \
  --workloads rs42_4K_ver,rs104_64K_ver,rs42_64K_enc,rs84_64K_enc,rs104_64K_enc,rs104_64K_rec2p_out \
  > "$OUT/trace.log" 2>&1
find "$OUT" -name '*stats*.csv'
