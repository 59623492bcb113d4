#!/bin/bash
# The per-object IEcDriver drop-in against the CPU codec, by object size (DESIGN.md
# §6): 4 KiB (configs[1]), 10 / 100 / 800 KiB (benchmark/k6/benchmark.js:14-19) and
# 1500 KiB (benchmark/go-ycsb/db/hybridstore/db.go:56); RS(4+2), 50/50 Encode /
# 1-erasure Reconstruct per call, DRAM-resident objects (each thread cycles through
# its share of ROTATE_MB MiB).  Per size:
#   * the CPU codec (oracle/ C restatement of klauspost's AVX-512 GFNI kernels),
#     one call per thread: 1 core, and the box's CPU quota;
#   * the coalesced GPU drop-in on caller memory (staged): 64 blocking callers, and
#     one event loop per quota core with 64 asynchronous calls in flight;
#   * the same two in place, objects in an rs_host_alloc arena (REGISTER=2);
#   * the Go shim's hybrid dispatch on arena objects (tools/run_hybrid.sh sweeps it).
# Callers are pinned to the quota's cores on the GPU's NUMA node.  One JSON line per
# run (tools/coalesce_bench.cpp); tools/coalesce_table.py makes the table.
# Usage: tools/run_drop_in.sh     (SIZES, SECS, ROTATE_MB override the defaults)
set -o pipefail
B=tools/coalesce_bench
run() {  # each run under its own limit; a limit, kill or fault (>= 124) ends the sweep
  echo "# REGISTER=${REGISTER:-0} $*" >&2
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
ONE="taskset -c ${CPUS%%-*}"
echo "# callers on cpus $CPUS, quota $Q" >&2
for OBJ in ${SIZES:-4096 10240 102400 819200 1536000}; do
  run $ONE $B 1 $SECS mix cpu 0 0 $OBJ
  run $PIN $B $Q $SECS mix cpu 0 0 $OBJ
  for R in 0 2; do
    REGISTER=$R run $PIN $B 64 $SECS mix co 0 0 $OBJ
    REGISTER=$R run $PIN $B $Q $SECS mix async 0 0 $OBJ 0 0 0 64
  done
  # the Go shim's hybrid dispatch on arena objects: the GPU for objects of >= 64 KiB
  # while fewer than 64 calls are there, the CPU codec for everything else
  # (integration/go/internal/ec/ec_gpu.go gpuMinObject / gpuMaxInflight)
  REGISTER=2 GPU_LIMIT=64 MIN_OBJ=65536 run $PIN $B $Q $SECS mix hybrid 0 0 $OBJ 0 0 0 6
done
