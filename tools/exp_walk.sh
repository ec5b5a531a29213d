#!/bin/bash
# A/B of index-build library variants (tools/build_variant.py dirs), bit-exact check included.
# usage (on the box): bash tools/exp_walk.sh SIZE REPS dir1 dir2 ...
set -o pipefail
N=$1; shift; R=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  HZ_LIB_VARIANT=$v timeout -k 10 150 python tools/debug/index_ab.py $N $R > gpurun_out/exw_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/exw_$v.log; exit 3; }
  tail -1 gpurun_out/exw_$v.log
done
