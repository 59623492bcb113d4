#!/bin/bash
# Direct per-object calls vs the coalescer (zero-copy staging, then staged DMA) at
# several caller counts; 4 KiB RS(4+2) objects.  args: threads secs wl mode max_batch
# max_wait obj max_exec staged_dma
set -e -o pipefail
B=tools/coalesce_bench
for wl in enc mix; do
  for T in 1 4 16 64 256; do
    timeout -k 5 60 $B $T 2 $wl direct
    timeout -k 5 60 $B $T 2 $wl co 4096 0 4096 0 0
    timeout -k 5 60 $B $T 2 $wl co 4096 0 4096 0 1
  done
done
for ex in 1 4; do timeout -k 5 60 $B 64 2 mix co 4096 0 4096 $ex 0; done
# larger objects: 64 KiB and 1 MiB (config 1's object size)
for obj in 65536 1048576; do
  for T in 1 16 64; do
    timeout -k 5 60 $B $T 2 enc direct 0 0 $obj
    timeout -k 5 60 $B $T 2 enc co 4096 0 $obj 0 0
  done
done
