#!/bin/bash
# Effective shader clock per dispatch under sustained back-to-back launches:
# GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) / kernel duration (MI355X_MICROARCH.md
# "DVFS give-back").  One rocprofv3 --pmc pass with the kernel trace per workload.
# Usage: tools/profile_clock.sh <tag> <iters> <workload>...
set -euo pipefail
TAG=$1; IT=$2; shift 2
export TMPDIR=/tmp
for W in "$@"; do
  OUT=gpurun_out/clk_${TAG}/$W
  mkdir -p "$OUT"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE -f csv -d "$OUT" -o run -- \
    python3 tools/ab_bench.py --rounds 1 --iters $IT --bpc 0 --workloads $W > "$OUT/log" 2>&1
  python3 tools/clock_summary.py "$OUT" rs::
done
