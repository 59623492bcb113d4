#!/bin/bash
# Caller wait policy A/B (rs_coalescer_opts.spin_waiters via SPIN): 4 KiB RS(4+2)
# 50/50 Encode / 1-erasure Reconstruct, blocking callers pinned to the CPU quota's
# cores, then one direct-call and one async reference line.  One JSON line per run.
set -o pipefail
B=tools/coalesce_bench
run() {
  echo "# SPIN=${SPIN:-0} $*" >&2
  timeout -k 5 60 "$@"
  local rc=$?
  if [ $rc -ge 124 ]; then exit $rc; fi
}
Q=$(awk '{if ($1 != "max") print int($1 / $2)}' /sys/fs/cgroup/cpu.max 2>/dev/null || true)
Q=${Q:-16}
PIN="taskset -c 0-$((Q - 1))"
for S in ${SPINS:-0 4 12}; do
  for T in ${CALLERS:-16 64 256}; do
    SPIN=$S run $PIN $B $T 2 mix co 0 0 ${OBJ:-4096}
  done
done
