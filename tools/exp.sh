#!/bin/bash
# Development A/B: GPU tests (optional) then bench lines under several env settings.
# usage (on the box): bash tools/exp.sh TAG [tests] -- "ENV=.. ENV2=.." "ENV=.." ...
set -o pipefail
T=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$1" = "tests" ]; then
  shift
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/exp_${T}_tests.log 2>&1 || { tail -30 gpurun_out/exp_${T}_tests.log; exit 2; }
  tail -2 gpurun_out/exp_${T}_tests.log
fi
[ "$1" = "--" ] && shift
SIZE=${SIZE:-17179869184}
DIST=${DIST:-zipf}
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --size $SIZE --dist $DIST \
    > gpurun_out/exp_${T}_$i.json 2> gpurun_out/exp_${T}_$i.err || { echo "cfg $cfg failed"; tail -5 gpurun_out/exp_${T}_$i.err; exit 3; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/exp_${T}_$i.json'))
print('$cfg', '|', d['value'], 'GB/s', d['ms_per_step'], 'ms', d['kernel_ms'], d.get('roundtrip_bit_exact'))"
done
