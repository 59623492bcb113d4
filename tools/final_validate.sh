#!/bin/bash
# Final-tree evidence in three gpurun calls (each under the 20-minute call limit):
#   part a: GPU tests, smoke, the default bench line, rocprofv3 of the bench (trace +
#           FETCH_SIZE / WRITE_SIZE passes) and of the bench's own K/M sweep windows
#   part b: the >= 2 GiB tests, per-leg compute-free ceilings, and the 2-rank bench
#           rehearsal on the one GPU
#   part c: the per-object drop-in table and the survey grid
# Usage: tools/final_validate.sh <tag> a|b|c
set -o pipefail
T=$1
case $2 in
a)
  tools/gpustep.sh ${T}_gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
  tools/gpustep.sh ${T}_smoke 120 python -c "import __graft_entry__ as g; g.smoke()" && \
  tools/gpustep.sh ${T}_bench 300 python bench.py --json-out gpurun_out/${T}_bench.json && \
  tools/gpustep.sh ${T}_prof_bench 400 tools/profile_bench.sh $T && \
  tools/gpustep.sh ${T}_sweep 700 tools/profile_sweep.sh $T
  ;;
b)
  tools/gpustep.sh ${T}_large_tests 300 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 250 --timeout-method thread && \
  tools/gpustep.sh ${T}_ceiling 700 tools/ceiling_probe.sh $T && \
  RSGPU_BENCH_BACKEND=gloo tools/gpustep.sh ${T}_bench_gpus2 300 python -u bench.py --gpus 2 --steps 50 \
    --json-out gpurun_out/${T}_bench_gpus2.json
  ;;
c)
  tools/gpustep.sh ${T}_drop_in 500 tools/run_drop_in.sh && \
  tools/gpustep.sh ${T}_survey 600 tools/run_survey.sh
  ;;
esac
