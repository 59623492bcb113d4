#!/bin/bash
# A/B: staging copies with streaming stores (default) vs plain memcpy
# (PLAIN_COPY=1 -> rs_coalescer_opts.plain_copy), staged per-object calls on DRAM-resident heap objects
# (ROTATE_MB=1024), RS(4+2) mix, 64 blocking callers on the GPU's NUMA node,
# alternating A B A B per size.
set -o pipefail
B=tools/coalesce_bench
run() {
  echo "# PLAIN_COPY=${PLAIN_COPY:-0} $*" >&2
  timeout -k 5 90 "$@"
  local rc=$?
  if [ $rc -ge 124 ]; then exit $rc; fi
}
Q=$(awk '{if ($1 != "max") print int($1 / $2)}' /sys/fs/cgroup/cpu.max 2>/dev/null || true)
Q=${Q:-16}
CPUS=$(tools/gpu_local_cpus.sh $Q)
PIN="taskset -c $CPUS"
export ROTATE_MB=1024
for OBJ in ${SIZES:-102400 819200 1536000}; do
  for rep in 1 2; do
    for PC in 0 1; do
      PLAIN_COPY=$PC run $PIN $B 64 2 mix co 0 0 $OBJ
    done
  done
done
