#!/bin/bash
# One step of a gpurun call: tools/gpustep.sh <name> <seconds> <command...>
# Output goes to gpurun_out/<name>.log.  A plain failure (exit < 124, e.g. a failing
# test) lets the chain go on; a time limit, kill, abort or fault (exit >= 124) makes
# this step fail so that `a && b && c` starts nothing more on the GPU.
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "$name rc=$rc"
[ "$rc" -lt 124 ]
