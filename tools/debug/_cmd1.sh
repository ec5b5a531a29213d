set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HZ_LIB_VARIANT=lib_segdbg timeout -k 10 120 python tools/debug/seg_debug.py 1048577 > gpurun_out/segdbg_1m.log 2>&1
grep -v amdgpu.ids gpurun_out/segdbg_1m.log | head -5
bash tools/gpu_quick.sh d "tests/test_gpu_extract.py tests/test_gpu_ranges.py" || exit 2
for v in lib lib_regwin; do
  HZ_LIB_VARIANT=$v timeout -k 10 200 python tools/debug/extract_loop.py 17179869184 2 zipf --only-indexless > gpurun_out/xloop_$v.log 2>&1 || { tail -5 gpurun_out/xloop_$v.log; exit 4; }
  echo "$v: $(grep rep gpurun_out/xloop_$v.log | tr '\n' ' ')"
done
for v in lib lib_hd2 lib_histold; do
  HZ_LIB_VARIANT=$v timeout -k 10 200 python tools/debug/stage_loop.py 17179869184 3 zipf h > gpurun_out/hloop_$v.log 2>&1 || { tail -5 gpurun_out/hloop_$v.log; exit 5; }
  echo "$v: $(grep 'rep 2' gpurun_out/hloop_$v.log)"
done
