set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HZ_LIB_VARIANT=lib_segdbg timeout -k 10 120 python tools/debug/seg_debug.py 1048577 > gpurun_out/segdbg_1m.log 2>&1
HZ_LIB_VARIANT=lib_segdbg timeout -k 10 120 python tools/debug/seg_debug.py 65541 >> gpurun_out/segdbg_1m.log 2>&1
cat gpurun_out/segdbg_1m.log | tail -20
bash tools/gpu_quick.sh c "tests/test_gpu_ranges.py tests/test_gpu.py"
