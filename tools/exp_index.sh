#!/bin/bash
# Development A/B of the index build: stage_loop's index stage under library variants / env settings.
# usage (on the box): bash tools/exp_index.sh TAG SIZE "ENV=.." "ENV=.." ...
set -o pipefail
T=$1; shift; N=$1; shift
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python tools/debug/stage_loop.py $N 3 zipf i > gpurun_out/exi_$T.log 2>&1 || { echo "cfg $cfg failed"; tail -5 gpurun_out/exi_$T.log; exit 3; }
  echo "$cfg | $(grep '^rep' gpurun_out/exi_$T.log | sed 's/.*index//' | tr '\n' ' ')"
done
