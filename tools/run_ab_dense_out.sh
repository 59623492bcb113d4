#!/bin/bash
# A/B: bounded out-of-place reconstructs writing into m rows per stripe (the full
# layout, only `bound` rows written: sparse writes) vs only `bound` rows per stripe
# (dense: stripe outputs back to back).  Two processes, each full then dense per
# workload, >= 100 ms of launches per round.
set -o pipefail
W=rs104_64K_rec1pb_out,rs104_64K_rec2pb_out,rs84_64K_rec1pb_out,rs84_64K_rec2pb_out,rs42_64K_rec1pb_out,rs42_4K_rec1pb_out
for pass in 1 2; do
  echo "== pass $pass"
  timeout -k 10 300 python -u tools/ab_bench.py --workloads $W --out-rows both --bpc 0 --rounds 3 --min-ms 100 || exit $?
done
