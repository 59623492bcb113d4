#!/bin/bash
# Interleaved A/B of abx/<variant>.so libraries on tools/ab_bench.py workloads.
# Usage: tools/run_ab.sh "<variants>" "<workloads>" [bpc list] [rounds]
set -euo pipefail
VARS=$1; WL=$2; BPC=${3:-0}; ROUNDS=${4:-2}
LIB=replication_erasurecoding_object_store_amd/librsgpu.so
cp $LIB /tmp/_librsgpu_keep.so
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    cp abx/$v.so $LIB
    echo "== round $r variant $v"
    timeout -k 10 240 python3 tools/ab_bench.py --rounds 1 --iters ${ITERS:-20} --bpc $BPC --workloads $WL ${AB_EXTRA:-} 2>&1 | grep -v amdgpu.ids
  done
done
cp /tmp/_librsgpu_keep.so $LIB
