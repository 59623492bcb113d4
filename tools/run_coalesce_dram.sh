#!/bin/bash
# Per-object CPU codec vs the coalesced GPU drop-in with DRAM-resident objects
# (ROTATE_MB=1024: every thread cycles through its share of 1 GiB of objects, 4x the
# host's L3) next to the cache-resident default.  RS(4+2), 50/50 Encode / 1-erasure
# Reconstruct; the CPU codec on 1 core and on the quota's cores, the GPU with 64
# blocking callers; all on the GPU's NUMA node.  One JSON line per run.
set -o pipefail
B=tools/coalesce_bench
run() {
  echo "# ROTATE_MB=${ROTATE_MB:-0} $*" >&2
  timeout -k 5 90 "$@"
  local rc=$?
  if [ $rc -ge 124 ]; then exit $rc; fi
}
Q=$(awk '{if ($1 != "max") print int($1 / $2)}' /sys/fs/cgroup/cpu.max 2>/dev/null || true)
Q=${Q:-16}
CPUS=$(tools/gpu_local_cpus.sh $Q)
PIN="taskset -c $CPUS"
ONE="taskset -c ${CPUS%%-*}"
for OBJ in ${SIZES:-4096 102400 1536000}; do
  for R in 0 1024; do
    ROTATE_MB=$R run $ONE $B 1 2 mix cpu 0 0 $OBJ
    ROTATE_MB=$R run $PIN $B $Q 2 mix cpu 0 0 $OBJ
    ROTATE_MB=$R run $PIN $B 64 2 mix co 0 0 $OBJ
  done
done
