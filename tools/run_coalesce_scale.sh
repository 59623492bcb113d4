#!/bin/bash
# Coalescer throughput vs concurrent callers: 4 KiB RS(4+2)
# objects, 50/50 Encode / 1-erasure Reconstruct, direct per-object calls vs the
# coalescer, 16..1024 caller threads.  One JSON line per run.  The GPU boxes give a
# 16-CPU cgroup quota (cpu.max) but a 256-CPU affinity mask: the pinned runs keep
# the process on as many cores as its quota (profiles/r02_coalesce_scale_pinned.log).
set -e -o pipefail
B=tools/coalesce_bench
Q=$(awk '{if ($1 != "max") print int($1 / $2)}' /sys/fs/cgroup/cpu.max 2>/dev/null || true)
for T in 16 64 256 1024; do
  timeout -k 5 60 $B $T 2 mix direct
  timeout -k 5 60 $B $T 2 mix co 4096 0 4096 0 0
  if [ -n "$Q" ]; then timeout -k 5 60 taskset -c 0-$((Q - 1)) $B $T 2 mix co 4096 0 4096 0 0; fi
done
