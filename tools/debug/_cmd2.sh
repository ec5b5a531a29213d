set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/gpu_tests_r04a.log 2>&1; rc=$?
tail -15 gpurun_out/gpu_tests_r04a.log
exit $rc
