#!/bin/bash
# Interleaved A/B of abx/<variant>.so libraries on tools/ab_bench.py workloads.
# Usage: tools/run_ab.sh "<variants>" "<workloads>" [bpc list] [rounds]
set -euo pipefail
VARS=$1; WL=$2; BPC=${3:-0}; ROUNDS=${4:-2}
# each variant is loaded by path (RSGPU_LIB): the shipped library is never replaced
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    echo "== round $r variant $v"
    RSGPU_LIB=$(pwd)/abx/$v.so timeout -k 10 240 python3 tools/ab_bench.py --rounds 1 --iters ${ITERS:-20} \
      --bpc $BPC --workloads $WL ${AB_EXTRA:-} 2>&1 | grep -v amdgpu.ids
  done
done
