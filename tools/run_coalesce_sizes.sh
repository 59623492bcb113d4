#!/bin/bash
# Per-object drop-in throughput at the reference's payload sizes:
# 4 KiB (configs[1]), 10 / 100 / 800 KiB (benchmark/k6/benchmark.js:14-19) and
# 1500 KiB (benchmark/go-ycsb/db/hybridstore/db.go:56), RS(4+2), 50/50 Encode /
# 1-erasure Reconstruct per call.  For each size: the CPU codec per call (oracle/
# C restatement of klauspost's AVX-512 GFNI kernels) on 1 core and on the box's CPU
# quota, then the coalesced GPU drop-in with 16 / 64 / 256 blocking callers on the
# quota's cores, then the asynchronous calls (rs_co_submit_* / rs_co_reap) from one
# event loop per quota core with DEPTHS calls in flight each.  One JSON line per run.
set -o pipefail
B=tools/coalesce_bench
# each run under its own time limit; a limit, kill or fault (>= 124) ends the sweep
run() {
  echo "# $*" >&2
  timeout -k 5 60 "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "# rc=$rc" >&2; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
}
SECS=${SECS:-2}
Q=$(awk '{if ($1 != "max") print int($1 / $2)}' /sys/fs/cgroup/cpu.max 2>/dev/null || true)
Q=${Q:-16}
# the quota's worth of cores on the GPU's NUMA node (where the pinned staging lives;
# node-0 cores run the large objects 17-21 % slower, profiles/r03h_coalesce_numa.log)
CPUS=$(tools/gpu_local_cpus.sh $Q)
PIN="taskset -c $CPUS"
ONE="taskset -c ${CPUS%%-*}"
echo "# callers on cpus $CPUS" >&2
for OBJ in ${SIZES:-4096 10240 102400 819200 1536000}; do
  run $ONE $B 1 $SECS mix cpu 0 0 $OBJ
  run $PIN $B $Q $SECS mix cpu 0 0 $OBJ
  for T in ${CALLERS:-16 64 256}; do
    run $PIN $B $T $SECS mix co 0 0 $OBJ
  done
  for D in ${DEPTHS:-16 64}; do
    run $PIN $B $Q $SECS mix async 0 0 $OBJ 0 0 0 $D
  done
done
