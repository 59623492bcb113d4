#!/bin/bash
# One box, one call: GPU tests, smoke, the default bench line, rocprofv3 trace + PMC
# of the bench (headline kernels) and of the K/M-sweep / config-3 workloads, so
# bench fractions and profiles/ summaries come from the same box.
# Usage: tools/gpu_validate.sh <tag>
set -o pipefail
T=$1
tools/gpustep.sh ${T}_gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
tools/gpustep.sh ${T}_smoke 120 python -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpustep.sh ${T}_bench 300 python bench.py && \
tools/gpustep.sh ${T}_prof_bench 600 tools/profile_bench.sh $T && \
tools/gpustep.sh ${T}_kmsweep_pmc 900 tools/profile_kmsweep_pmc.sh $T rs42_64K_enc rs42_64K_rec2p_out rs42_64K_rec1pb_out \
  rs84_64K_enc rs84_64K_rec2pb_out rs84_64K_rec1pb_out rs84_64K_rec2p_out rs84_64K_rec1p_out \
  rs104_64K_enc rs104_64K_rec2pb_out rs104_64K_rec1pb_out rs104_64K_rec2p_out rs104_64K_rec1p_out \
  rs42_4K_rec1pb_out rs42_4K_rec2u_out rs42_4K_rec04u_out rs42_4K_rec45u_out
