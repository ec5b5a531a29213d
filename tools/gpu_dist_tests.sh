set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/dist_tests.log 2>&1; rc=$?
tail -15 gpurun_out/dist_tests.log
exit $rc
