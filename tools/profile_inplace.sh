#!/bin/bash
# rocprofv3 kernel trace of the per-object drop-in with 1.5 MB objects in place
# (rs_host_alloc arena, REGISTER=2) and staged (heap objects): the pointer-table
# kernel's duration per batch against the bytes it moves over PCIe.
# Usage: tools/profile_inplace.sh <tag>
set -euo pipefail
TAG=$1
OUT=gpurun_out/inplace_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp ROTATE_MB=1024
Q=$(awk '{if ($1 != "max") print int($1 / $2)}' /sys/fs/cgroup/cpu.max 2>/dev/null || true)
CPUS=$(tools/gpu_local_cpus.sh ${Q:-16})
for R in 2 0; do
  REGISTER=$R timeout -k 10 120 taskset -c "$CPUS" rocprofv3 --kernel-trace --stats -f csv -d "$OUT/reg$R" -o run \
    -- tools/coalesce_bench 64 2 mix co 0 0 1536000 > "$OUT/reg$R.log" 2>&1
done
echo "done $TAG"
