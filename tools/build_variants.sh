#!/bin/bash
# build_variants.sh <name>:<kernel-source relative to the repo root>:<defines> ... : builds A/B variants of
# librsgpu.so into ab_libs/<name>.so (only rs_kernels*.hip differs; the other
# objects come from the normal build).  Used with tools/ab_libs.py --libs.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/replication_erasurecoding_object_store_amd/csrc
make -s -C "$CS"
mkdir -p "$ROOT/ab_libs"
FLAGS="-I$CS -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result"
OTHERS="$CS/build/rs_sha256.hip.o $CS/build/rs_engine.cpp.o $CS/build/rs_coalescer.cpp.o $CS/build/gf256.cpp.o"
for spec in "$@"; do
  IFS=: read -r name src defs <<<"$spec"
  /opt/rocm/bin/hipcc $FLAGS $defs -c "$ROOT/$src" -o "$ROOT/ab_libs/$name.o"
  /opt/rocm/bin/hipcc $FLAGS -shared -o "$ROOT/ab_libs/$name.so" "$ROOT/ab_libs/$name.o" $OTHERS
  rm -f "$ROOT/ab_libs/$name.o"
  echo "built ab_libs/$name.so"
done
