# device codebook / header GPU tests, the codebook phase profile (lib_cbprof variant), the device-vs-host latency
# comparison (tools/cb_latency.py) and its kernel trace (needs: python huffman_amd/build.py --variant cbprof -DHZ_CB_PROF)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_codebook.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t8_tests.log 2>&1; rc=$?
tail -3 gpurun_out/t8_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/t8_tests.log | head -30; exit $rc; }
HZ_LIB_VARIANT=lib_cbprof timeout -k 10 120 python tools/debug/cb_prof.py > gpurun_out/cbprof.log 2>&1 || { tail gpurun_out/cbprof.log; exit 9; }
grep -E "init|r  [0-9] " gpurun_out/cbprof.log
timeout -k 10 300 python -u tools/cb_latency.py --reps 11 --out gpurun_out/cb_latency.json > gpurun_out/t8_lat.log 2>&1 || { tail -20 gpurun_out/t8_lat.log; exit 7; }
grep -A2 '"device_codebook"' gpurun_out/cb_latency.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/t8_prof -o cbl --output-format csv -- python3 tools/cb_latency.py --reps 5 > gpurun_out/t8_prof.log 2>&1 || { tail -20 gpurun_out/t8_prof.log; exit 8; }
grep -hE "k_cb|k_hdr|k_header" gpurun_out/t8_prof/cbl_kernel_stats.csv | cut -d, -f1-4
