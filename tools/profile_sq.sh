#!/bin/bash
# SQ / SQC counters per A/B workload (tools/ab_bench.py), one rocprofv3 --pmc pass per
# counter group (gfx950 limits: 8 SQ counters per pass).
# Usage: tools/profile_sq.sh <tag> <workload>...
set -euo pipefail
TAG=$1; shift 1
export TMPDIR=/tmp
SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM"
SQ2="SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_IFETCH SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
for W in "$@"; do
  OUT=gpurun_out/sq_${TAG}/$W
  mkdir -p "$OUT"
  ARGS="--rounds 1 --iters 6 --bpc 0 --workloads $W"
  timeout -s KILL 90 rocprofv3 --pmc $SQ1 -f csv -d "$OUT/sq1" -o run -- python3 tools/ab_bench.py $ARGS > "$OUT/sq1.log" 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $SQ2 -f csv -d "$OUT/sq2" -o run -- python3 tools/ab_bench.py $ARGS > "$OUT/sq2.log" 2>&1 || echo "sq2 failed $W"
  echo "done $W"
done
