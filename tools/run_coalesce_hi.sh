#!/bin/bash
set -e -o pipefail
B=tools/coalesce_bench
for T in 64 256 1024; do
  timeout -k 5 60 $B $T 2 mix direct
  timeout -k 5 60 $B $T 2 mix co 4096 0 4096 0 0
done
