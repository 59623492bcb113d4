#!/bin/bash
# Coalescer diagnostics at high caller counts (RS_CO_DEBUG prints launcher
# straggler-wait, device-wait and back-pressure totals at destroy).
set -e -o pipefail
B=tools/coalesce_bench
for T in 64 256 1024; do
  RS_CO_DEBUG=1 timeout -k 5 60 $B $T 2 mix co 4096 0 4096 0 0
done
