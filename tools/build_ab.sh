#!/bin/bash
# A/B build: links librsgpu variants that differ only in the kernel translation
# unit (a source file and/or -D flags) into abx/<name>.so.  Experiment scaffolding:
# abx/ is git-ignored; run a variant by path (RSGPU_LIB=abx/<name>.so, or tools/ab_same.py).
# Usage: [ENGINE_FLAGS="-DX=1"] tools/build_ab.sh <name> <kernel.hip> [-DFLAG=...]
# (ENGINE_FLAGS: rs_engine.cpp is rebuilt with them for this variant only)
set -euo pipefail
NAME=$1; SRC=$2; shift 2
C=replication_erasurecoding_object_store_amd/csrc
make -s -C $C >/dev/null
mkdir -p abx
# a copy next to the sources (their includes), one per variant: builds may run in parallel
cp "$SRC" $C/_ab_$NAME.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result "$@" -c $C/_ab_$NAME.hip -o /tmp/_ab_$NAME.o
rm -f $C/_ab_$NAME.hip
ENG=$C/build/rs_engine.cpp.o
if [ -n "${ENGINE_FLAGS:-}" ]; then
  ENG=/tmp/_ab_${NAME}_engine.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result $ENGINE_FLAGS \
    -c $C/rs_engine.cpp -o $ENG
fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o abx/$NAME.so /tmp/_ab_$NAME.o \
  $C/build/rs_sha256.hip.o $ENG $C/build/rs_coalescer.cpp.o $C/build/gf256.cpp.o \
  $C/build/rs_host_copy.cpp.o
echo "abx/$NAME.so"
