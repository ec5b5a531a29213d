#!/bin/bash
# Kernel A/B on the GPU box: stage_loop.py under each library variant (HZ_LIB_VARIANT dirs), interleaved
# ROUNDS times so box drift hits every variant alike.
# usage: bash tools/ab.sh STAGES SIZE DIST ROUNDS dir1 dir2 ...   (dir "lib" = the product build)
set -o pipefail
ST=$1; SIZE=$2; DIST=$3; ROUNDS=$4; shift 4
mkdir -p gpurun_out
for r in $(seq 1 $ROUNDS); do
  for d in "$@"; do
    HZ_LIB_VARIANT=$d timeout -k 10 120 python tools/debug/stage_loop.py $SIZE 3 $DIST $ST > gpurun_out/ab_${d}_$r.log 2>&1 \
      || { echo "variant $d failed"; tail -5 gpurun_out/ab_${d}_$r.log; exit 3; }
    echo "$d r$r: $(grep '^rep 2' gpurun_out/ab_${d}_$r.log) $(tail -1 gpurun_out/ab_${d}_$r.log)"
  done
done
