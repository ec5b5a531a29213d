# walker: escape gather issued at the parking step (HZ_WALK_EARLY) vs at the resolve; correctness of the variant
set -o pipefail
mkdir -p gpurun_out
HZ_LIB_VARIANT=lib_early timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q -k "index" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t14_tests.log 2>&1; rc=$?
tail -2 gpurun_out/t14_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/t14_tests.log | head -30; exit $rc; }
bash tools/ab.sh i 17179869184 zipf 3 lib lib_early
