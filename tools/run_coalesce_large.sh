#!/bin/bash
# Large-object drop-in tuning sweep: 800 KiB and 1500 KiB RS(4+2) objects, 50/50
# Encode / 1-erasure Reconstruct, 64 blocking callers on the CPU quota's cores;
# batches executing at once (max_exec 2 / 4), zero-copy vs staged DMA, 32 vs
# 128 MiB of staging per batch (BATCH_MB).  One JSON line per run.
set -o pipefail
B=tools/coalesce_bench
run() {
  echo "# BATCH_MB=${BATCH_MB:-32} $*" >&2
  timeout -k 5 60 "$@"
  local rc=$?
  if [ $rc -ge 124 ]; then exit $rc; fi
}
Q=$(awk '{if ($1 != "max") print int($1 / $2)}' /sys/fs/cgroup/cpu.max 2>/dev/null || true)
Q=${Q:-16}
PIN="taskset -c 0-$((Q - 1))"
for OBJ in 819200 1536000; do
  for MB in 32 128; do
    for EX in 2 4; do
      for DMA in 0 1; do
        BATCH_MB=$MB run $PIN $B 64 2 mix co 0 0 $OBJ $EX $DMA 32
      done
    done
  done
done
