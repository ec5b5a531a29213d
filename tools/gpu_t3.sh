set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t3_tests.log 2>&1; rc=$?
tail -3 gpurun_out/t3_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/t3_tests.log | head -20; exit $rc; }
bash tools/ab.sh d 17179869184 zipf 2 lib_base lib
