set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HZ_LIB_VARIANT=lib_segdbg timeout -k 10 120 python tools/debug/seg_debug.py 1048577 > gpurun_out/segdbg_1m.log 2>&1
grep -v amdgpu.ids gpurun_out/segdbg_1m.log | head -5
bash tools/gpu_quick.sh d "tests/test_gpu_extract.py tests/test_gpu_ranges.py tests/test_gpu.py" || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_d -o run --output-format csv -- python3 tools/debug/extract_loop.py 17179869184 2 > gpurun_out/xloop_d.log 2>&1 || { tail -5 gpurun_out/xloop_d.log; exit 4; }
cat gpurun_out/xloop_d.log | grep -v amdgpu.ids
find gpurun_out/prof_d -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-4 {} | head -25'
