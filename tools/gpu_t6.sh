# default (count + scan + write) GPU tests, the opt-in one-pass pack's test, and a 16 GiB pack A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_gpu_codebook.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t6_tests.log 2>&1; rc=$?
tail -3 gpurun_out/t6_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/t6_tests.log | head -20; exit $rc; }
for v in 0 1; do
  HZ_PACK_LB=$v timeout -k 10 120 python tools/debug/stage_loop.py 17179869184 3 zipf p > gpurun_out/t6_ab_${v}.log 2>&1 || exit 6
  echo "LB=$v: $(grep '^rep 2' gpurun_out/t6_ab_${v}.log) $(tail -1 gpurun_out/t6_ab_${v}.log)"
done
