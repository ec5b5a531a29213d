#!/bin/bash
# GPU check used during development: probe one file, GPU tests, 4 GiB and 16 GiB Zipf bench.
# usage (on the box): bash tools/gpu_check.sh TAG
set -o pipefail
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 python tools/debug/stage_probe.py tests/golden/romeo.txt.compressed > gpurun_out/probe_$T.log 2>&1 || exit 1
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests_$T.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 1 --size 4294967296 > gpurun_out/b_${T}_4g.json 2> gpurun_out/b_$T.err || exit 3
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/b_${T}_zipf.json 2>> gpurun_out/b_$T.err || exit 4
