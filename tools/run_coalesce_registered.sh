#!/bin/bash
# Per-object drop-in with the objects in a registered arena (REGISTER=1) or an
# rs_host_alloc arena (REGISTER=2) -- coalesced
# calls run in place, no staging copies) vs heap objects (staged), DRAM-resident
# (ROTATE_MB=1024), RS(4+2) 50/50 Encode / 1-erasure Reconstruct; 64 blocking callers
# and 16 async loops x 16 in flight on the GPU's NUMA node, the CPU codec on one core
# of it beside.  One JSON line per run.
set -o pipefail
B=tools/coalesce_bench
run() {
  echo "# REGISTER=${REGISTER:-0} ROTATE_MB=${ROTATE_MB:-0} $*" >&2
  timeout -k 5 90 "$@"
  local rc=$?
  if [ $rc -ge 124 ]; then exit $rc; fi
}
Q=$(awk '{if ($1 != "max") print int($1 / $2)}' /sys/fs/cgroup/cpu.max 2>/dev/null || true)
Q=${Q:-16}
CPUS=$(tools/gpu_local_cpus.sh $Q)
PIN="taskset -c $CPUS"
export ROTATE_MB=1024
for OBJ in ${SIZES:-4096 102400 819200 1536000}; do
  run taskset -c ${CPUS%%-*} $B 1 2 mix cpu 0 0 $OBJ
  for R in ${REGS:-0 1 2}; do
    REGISTER=$R run $PIN $B 64 2 mix co 0 0 $OBJ
    REGISTER=$R run $PIN $B $Q 2 mix async 0 0 $OBJ 0 0 0 16
  done
done
