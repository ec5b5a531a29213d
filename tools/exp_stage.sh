#!/bin/bash
# Timing A/B of one stage under env settings via tools/debug/stage_loop.py (no bit-exact check implied).
# usage (on the box): bash tools/exp_stage.sh TAG "ARGS" "ENV=.." "ENV=.." ...
set -o pipefail
T=$1; shift; A=$1; shift
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python tools/debug/stage_loop.py $A > gpurun_out/exs_$T.log 2>&1 || { echo "cfg $cfg failed"; tail -5 gpurun_out/exs_$T.log; exit 3; }
  echo "$cfg | $(tail -2 gpurun_out/exs_$T.log | tr '\n' ' ')"
done
