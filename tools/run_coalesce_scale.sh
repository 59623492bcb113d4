#!/bin/bash
# Coalescer throughput vs concurrent callers: 4 KiB RS(4+2)
# objects, 50/50 Encode / 1-erasure Reconstruct, direct per-object calls vs the
# coalescer, 16..1024 caller threads.  One JSON line per run.
set -e -o pipefail
B=tools/coalesce_bench
for T in 16 64 256 1024; do
  timeout -k 5 60 $B $T 2 mix direct
  timeout -k 5 60 $B $T 2 mix co 4096 0 4096 0 0
done
