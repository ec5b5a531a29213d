#!/bin/bash
# One rocprofv3 counter pass per argument group over tools/debug/stage_loop.py.
# usage (on the box): bash tools/pmc_pass.sh TAG "ARGS for stage_loop" "CTR CTR .." "CTR .." ...
set -o pipefail
T=$1; shift; A=$1; shift
O=gpurun_out/pmc_$T; mkdir -p $O
export TMPDIR=/tmp
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $O/p$i -o run --output-format csv -- python3 tools/debug/stage_loop.py $A \
    > $O/p$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -5 $O/p$i.log; exit 3; }
done
python3 tools/pmc_summary.py $O
