set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/op_tests.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/op_b1.json 2> gpurun_out/op_b1.err && \
HZ_PACK_ONEPASS=0 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/op_b0.json 2> gpurun_out/op_b0.err
