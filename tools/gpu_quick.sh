#!/bin/bash
# Development GPU check (on the box, repo root): selected GPU tests, then the 16 GiB Zipf bench.
# usage: bash tools/gpu_quick.sh TAG "pytest -k expression or test paths"
set -o pipefail
T=${1:-x}; SEL=${2:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/q_tests_$T.log 2>&1 || { tail -30 gpurun_out/q_tests_$T.log; exit 2; }
tail -3 gpurun_out/q_tests_$T.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/q_bench_$T.json 2> gpurun_out/q_bench_$T.err \
  || { tail -20 gpurun_out/q_bench_$T.err; exit 3; }
python - <<PY
import json
d=json.load(open("gpurun_out/q_bench_$T.json"))
print({k: d[k] for k in ("value","ms_per_step","roundtrip_bit_exact","kernel_ms")}, "enc_frac", d["encode_roofline"]["frac"], "enc_ms", d["encode_roofline"]["ms"], d["index_build_from_payload"], d["extract_indexless"])
PY
