#!/bin/bash
# A/B: out-of-place reconstructs with and without rs_set_out_pad_writes (output rows
# written to whole 128-B lines), interleaved in one process, two processes.
set -o pipefail
W=rs104_64K_rec1pb_out,rs104_64K_rec2pb_out,rs104_64K_rec2p_out,rs84_64K_rec2pb_out,rs42_4K_rec2p_out
for pass in 1 2; do
  echo "== pass $pass"
  timeout -k 10 300 python -u tools/ab_bench.py --workloads $W --out-pad both --bpc 0 --rounds 3 --min-ms 100 || exit $?
done
