#!/bin/bash
# Direct vs coalesced per-object calls at several caller counts (4 KiB objects).
set -e -o pipefail
B=tools/coalesce_bench
for wl in enc mix; do
  for T in 1 4 16 64 256; do
    timeout -k 5 60 $B $T 3 $wl direct
    timeout -k 5 60 $B $T 3 $wl co 4096 0
  done
done
# execution concurrency and linger at 64 callers
for ex in 1 2 4; do timeout -k 5 60 $B 64 3 mix co 4096 0 4096 $ex; done
timeout -k 5 60 $B 64 3 mix co 4096 50
