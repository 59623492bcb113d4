#!/bin/bash
# Hybrid CPU/GPU dispatch of the per-object drop-in, by
# object size: RS(4+2), 50/50 Encode / 1-erasure Reconstruct per call, DRAM-resident
# objects, callers pinned to the box's CPU quota on the GPU's NUMA node.  Per size:
#   * CPU only: the CPU codec (oracle/'s C restatement of klauspost's GFNI kernels,
#     standing in for klauspost -- measurement only, never in the product), one call
#     per thread on every quota core;
#   * GPU only: the coalescer's asynchronous calls, one event loop per quota core
#     with 64 calls in flight (the Go shim's model);
#   * hybrid: the same loops, but an object goes to the GPU only while fewer than
#     GPU_LIMIT calls are in flight there (and on RS_ERR_BUSY it runs on the CPU),
#     every other object on the CPU codec on the loop's thread; MIN_OBJ: objects
#     below it never go to the GPU.
# One JSON line per run (tools/coalesce_bench.cpp); tools/coalesce_table.py makes
# the table.  Usage: tools/run_hybrid.sh  (SIZES, SECS, LIMITS, MIN_OBJ override)
set -o pipefail
B=tools/coalesce_bench
run() {  # each run under its own limit; a limit, kill or fault (>= 124) ends the sweep
  echo "# REGISTER=${REGISTER:-0} GPU_LIMIT=${GPU_LIMIT:-} MIN_OBJ=${MIN_OBJ:-} $*" >&2
  timeout -k 5 60 "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "# rc=$rc" >&2; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
}
SECS=${SECS:-2}
export ROTATE_MB=${ROTATE_MB:-1024}
Q=$(awk '{if ($1 != "max") print int($1 / $2)}' /sys/fs/cgroup/cpu.max 2>/dev/null || true)
Q=${Q:-16}
CPUS=$(tools/gpu_local_cpus.sh $Q)
PIN="taskset -c $CPUS"
echo "# callers on cpus $CPUS, quota $Q" >&2
# REGISTER=2: the objects live in an rs_host_alloc arena, so GPU calls run in place
# (no staging copy on the CPU); the CPU codec works on the same memory
for OBJ in ${SIZES:-4096 10240 102400 819200 1536000}; do
  run $PIN $B $Q $SECS mix cpu 0 0 $OBJ
  for R in ${REGS:-0 2}; do
    REGISTER=$R run $PIN $B $Q $SECS mix async 0 0 $OBJ 0 0 0 64
    for L in ${LIMITS:-16 64}; do
      D=$(( L / Q + 2 ))
      REGISTER=$R GPU_LIMIT=$L MIN_OBJ=${MIN_OBJ:-0} run $PIN $B $Q $SECS mix hybrid 0 0 $OBJ 0 0 0 $D
    done
  done
done
