#!/bin/bash
# A/B build: links librsgpu variants that differ only in the kernel translation
# unit (a source file and/or -D flags) into abx/<name>.so.  Experiment scaffolding:
# abx/ is git-ignored; run a variant by copying it over the in-tree librsgpu.so.
# Usage: tools/build_ab.sh <name> <kernel.hip> [-DFLAG=...]
set -euo pipefail
NAME=$1; SRC=$2; shift 2
C=replication_erasurecoding_object_store_amd/csrc
make -s -C $C >/dev/null
mkdir -p abx
# a copy next to the sources (their includes), one per variant: builds may run in parallel
cp "$SRC" $C/_ab_$NAME.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result "$@" -c $C/_ab_$NAME.hip -o /tmp/_ab_$NAME.o
rm -f $C/_ab_$NAME.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o abx/$NAME.so /tmp/_ab_$NAME.o \
  $C/build/rs_sha256.hip.o $C/build/rs_engine.cpp.o $C/build/rs_coalescer.cpp.o $C/build/gf256.cpp.o \
  $C/build/rs_host_copy.cpp.o
echo "abx/$NAME.so"
