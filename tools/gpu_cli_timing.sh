# GPU tests of test_gpu.py (the CLIs among them), then the 16 GiB CLI stage split (tools/cli_timing.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t10_tests.log 2>&1; rc=$?
tail -3 gpurun_out/t10_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/t10_tests.log | head -30; exit $rc; }
timeout -k 10 600 python -u tools/cli_timing.py --gib 16 --out gpurun_out/r03d_cli_timing_16g.json > gpurun_out/t10_cli.log 2>&1 || { tail gpurun_out/t10_cli.log; exit 6; }
python -c "import json;d=json.load(open('gpurun_out/r03d_cli_timing_16g.json'));print({k:{x:d[k][x] for x in ('total_ms','fread_ms','fwrite_ms','alloc_ms','host_ms','kernel_ms','process_wall_s')} for k in ('archive','extract')}, d['round_trip_identical'])"
