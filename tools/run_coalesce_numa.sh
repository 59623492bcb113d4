#!/bin/bash
# Caller placement vs the GPU's NUMA node: the coalescer's pinned staging lives on
# the GPU's node (rs_engine.cpp device_numa_node); callers pinned to the quota's
# worth of cores on node 0 (cpus 0-15) and on the GPU's node (first cores of the
# node rs_backend reports).  RS(4+2), 50/50 Encode / 1-erasure Reconstruct, 64
# blocking callers, 4 KiB / 800 KiB / 1500 KiB objects; CPU codec on 1 core beside.
set -o pipefail
B=tools/coalesce_bench
run() {
  echo "# $*" >&2
  timeout -k 5 60 "$@"
  local rc=$?
  if [ $rc -ge 124 ]; then exit $rc; fi
}
Q=$(awk '{if ($1 != "max") print int($1 / $2)}' /sys/fs/cgroup/cpu.max 2>/dev/null || true)
Q=${Q:-16}
NODE=$(python3 -c "
import sys; sys.path.insert(0, '.')
from replication_erasurecoding_object_store_amd import _lib
import ctypes
L = _lib.lib(); ctx = ctypes.c_void_p()
assert L.rs_create(4, 2, 0, 0, ctypes.byref(ctx)) == 0
b = L.rs_backend(ctx).decode(); L.rs_destroy(ctx)
print(b.split('numa')[-1])")
FIRST=$(awk -v n="$NODE" -F'[ ,-]+' '$0 ~ "NUMA node"n" CPU" {print $4}' <(lscpu))
echo "# GPU numa node $NODE, first cpu $FIRST" >&2
for OBJ in 4096 819200 1536000; do
  run taskset -c "$FIRST" $B 1 2 mix cpu 0 0 $OBJ
  for CPUS in "0-$((Q - 1))" "$FIRST-$((FIRST + Q - 1))"; do
    run taskset -c $CPUS $B 64 2 mix co 0 0 $OBJ
  done
done
