# device codebook / header tests, then the latency comparison and a kernel trace of it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_codebook.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t7_tests.log 2>&1; rc=$?
tail -3 gpurun_out/t7_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/t7_tests.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/cb_latency.py --reps 11 --out gpurun_out/cb_latency.json > gpurun_out/t7_lat.log 2>&1 || { tail -20 gpurun_out/t7_lat.log; exit 7; }
cat gpurun_out/cb_latency.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/t7_prof -o cbl --output-format csv -- python3 tools/cb_latency.py --reps 5 > gpurun_out/t7_prof.log 2>&1 || { tail -20 gpurun_out/t7_prof.log; exit 8; }
find gpurun_out/t7_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} grep -E "k_codebook|k_hdr|k_header" {}
