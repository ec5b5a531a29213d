set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ranges.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/q13.log 2>&1 || { tail -30 gpurun_out/q13.log; exit 2; }
tail -2 gpurun_out/q13.log
for v in lib; do
  HZ_LIB_VARIANT=$v timeout -k 10 200 python tools/debug/stage_loop.py 17179869184 4 zipf p > gpurun_out/ploop_$v.log 2>&1 || { tail -5 gpurun_out/ploop_$v.log; exit 5; }
  echo "$v: $(grep -E 'rep (2|3)' gpurun_out/ploop_$v.log | grep -oE "'pack': [0-9.]+" | tr '\n' ' ')"
done
