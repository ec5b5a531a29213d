# round-end checks: full GPU suite, smoke, 16 GiB CLI timing
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r04h.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r04h.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/gpu_tests_r04h.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r04h.log 2>&1 || { tail -20 gpurun_out/smoke_r04h.log; exit 3; }
tail -1 gpurun_out/smoke_r04h.log
timeout -k 10 600 python -u tools/cli_timing.py --gib 16 --out gpurun_out/r04h_cli_timing_16g.json > gpurun_out/cli_r04h.log 2>&1 || { tail gpurun_out/cli_r04h.log; exit 6; }
python -c "import json;d=json.load(open('gpurun_out/r04h_cli_timing_16g.json'));print({k:{x:d[k][x] for x in ('total_ms','fread_ms','fwrite_ms','alloc_ms','host_ms','kernel_ms','process_wall_s')} for k in ('archive','extract')}, d['round_trip_identical'])"
