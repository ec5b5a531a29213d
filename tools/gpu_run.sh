#!/bin/bash
# One GPU call, several steps (on the box, repo root): each step under its own time limit; the call
# stops at the first failing step (no further GPU work after a failure, a timeout or a fault).
# usage: bash tools/gpu_run.sh TAG "step 1" "step 2" ...
set -o pipefail
T=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for step in "$@"; do
  i=$((i + 1))
  echo "[gpu_run $T] step $i: $step"
  bash -c "$step" > gpurun_out/${T}_s$i.log 2>&1
  rc=$?
  tail -4 gpurun_out/${T}_s$i.log
  if [ $rc -ne 0 ]; then echo "[gpu_run $T] step $i failed rc=$rc"; exit $rc; fi
done
echo "[gpu_run $T] all $i steps ok"
