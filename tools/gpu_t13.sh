# index tests, then index build A/B (walker table with unambiguous long prefixes vs base)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q -k "index or extract or decode or file or stream" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t13_tests.log 2>&1; rc=$?
tail -2 gpurun_out/t13_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/t13_tests.log | head -30; exit $rc; }
bash tools/ab.sh i 17179869184 zipf 3 lib_base lib
