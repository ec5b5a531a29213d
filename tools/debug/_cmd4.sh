set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HZ_LIB_VARIANT=lib_segdbg timeout -k 10 120 python tools/debug/seg_debug.py 1048577 > gpurun_out/segdbg_1m.log 2>&1 || { tail -20 gpurun_out/segdbg_1m.log; exit 1; }
grep -v amdgpu.ids gpurun_out/segdbg_1m.log | head -12
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/q_tests_x.log 2>&1 || { tail -30 gpurun_out/q_tests_x.log; exit 2; }
tail -2 gpurun_out/q_tests_x.log
for v in lib; do
  HZ_LIB_VARIANT=$v timeout -k 10 200 python tools/debug/extract_loop.py 17179869184 2 zipf --only-indexless > gpurun_out/xloop_$v.log 2>&1 || { tail -5 gpurun_out/xloop_$v.log; exit 4; }
  echo "$v: $(grep rep gpurun_out/xloop_$v.log | tr '\n' ' ')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/xprof -o xprof --output-format csv -- python3 tools/debug/extract_loop.py 17179869184 2 zipf --only-indexless > gpurun_out/xprof.log 2>&1 || { tail -20 gpurun_out/xprof.log; exit 5; }
f=$(find gpurun_out/xprof -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -12
