#!/bin/bash
# isa_stats.sh <asm.s> <mangled-kernel-name>... : static instruction mix of kernels
# (produce the .s with: hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S rs_kernels.hip -o k.s)
s=$1; shift
for f in "$@"; do
  awk -v f="$f:" 'index($0,f)==1{p=1} p{print} p&&/s_endpgm/{exit}' "$s" > /tmp/_isa_one.s
  echo "$f lines=$(wc -l </tmp/_isa_one.s) valu=$(grep -cE '^\s+v_' /tmp/_isa_one.s) perm=$(grep -c v_perm /tmp/_isa_one.s)" \
       "bitop3=$(grep -c v_bitop3 /tmp/_isa_one.s) vmov=$(grep -c v_mov /tmp/_isa_one.s) sload=$(grep -c s_load /tmp/_isa_one.s)" \
       "readlane=$(grep -c readlane /tmp/_isa_one.s) writelane=$(grep -c writelane /tmp/_isa_one.s)" \
       "and=$(grep -c v_and_b32 /tmp/_isa_one.s) shr=$(grep -c v_lshrrev /tmp/_isa_one.s) waitcnt=$(grep -c s_waitcnt /tmp/_isa_one.s)"
done
