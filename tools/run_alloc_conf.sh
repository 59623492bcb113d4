#!/bin/bash
# Per-process spread vs how torch maps device memory: the same legs in alternating
# processes with the default caching allocator and with expandable segments
# (PYTORCH_HIP_ALLOC_CONF=expandable_segments:True), two processes each.
set -o pipefail
W=rs104_64K_rec1pb_out,rs104_64K_enc,rs42_4K_rec2p_out
for pass in 1 2; do
  for conf in default expandable; do
    echo "== pass $pass $conf"
    if [ $conf = expandable ]; then
      PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 200 python -u tools/ab_bench.py --workloads $W --bpc 0 --rounds 3 --min-ms 100 || exit $?
    else
      timeout -k 10 200 python -u tools/ab_bench.py --workloads $W --bpc 0 --rounds 3 --min-ms 100 || exit $?
    fi
  done
done
