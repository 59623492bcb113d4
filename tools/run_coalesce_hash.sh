#!/bin/bash
# The write path's Encode + cold_hash per object (rs_co_encode_hash), DRAM-resident
# objects (ROTATE_MB=1024), RS(4+2): staged heap objects (REGISTER=0) vs objects in
# an rs_host_alloc arena (REGISTER=2: encode and hash in place), 64 blocking callers
# on the GPU's NUMA node, beside the CPU codec + SHA-NI on one core of it.
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
for OBJ in ${SIZES:-4096 10240 102400 819200 1536000}; do
  run taskset -c ${CPUS%%-*} $B 1 2 hash cpu 0 0 $OBJ
  for R in 0 2; do
    REGISTER=$R run $PIN $B 64 2 hash co 0 0 $OBJ
    REGISTER=$R run $PIN $B 64 2 enc co 0 0 $OBJ
  done
done
