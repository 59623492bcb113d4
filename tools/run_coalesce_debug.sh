#!/bin/bash
# Coalescer diagnostics at high caller counts (CO_TIMING prints the launcher's
# straggler-wait, device-wait and back-pressure totals from rs_co_timing).
set -e -o pipefail
B=tools/coalesce_bench
for T in 64 256 1024; do
  CO_TIMING=1 timeout -k 5 60 $B $T 2 mix co 4096 0 4096 0 0
done
