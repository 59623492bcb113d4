#!/bin/bash
# In-place 1.5 MB objects (rs_host_alloc arena, DRAM-resident): batches executing at
# once (max_exec) and staging bytes per batch (BATCH_MB: in-place slots still take
# a slot's share of it), blocking callers; the device idles 37 % of the time at the
# defaults (profiles/r03z_prof_inplace.md).
set -o pipefail
B=tools/coalesce_bench
run() {
  echo "# REGISTER=${REGISTER:-0} BATCH_MB=${BATCH_MB:-32} $*" >&2
  timeout -k 5 90 "$@"
  local rc=$?
  if [ $rc -ge 124 ]; then exit $rc; fi
}
Q=$(awk '{if ($1 != "max") print int($1 / $2)}' /sys/fs/cgroup/cpu.max 2>/dev/null || true)
Q=${Q:-16}
CPUS=$(tools/gpu_local_cpus.sh $Q)
PIN="taskset -c $CPUS"
export ROTATE_MB=1024 REGISTER=2
for rep in 1 2; do
  for MB in 32 64 128; do
    for EX in 2 4; do
      BATCH_MB=$MB run $PIN $B 64 2 mix co 0 0 1536000 $EX 0 16
    done
  done
done
