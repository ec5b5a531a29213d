# full GPU test suite (device codebook in archive, device header parse in extract), then the CLI
# stage split at 1 GiB with the device and the host codebook/header paths
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t9_tests.log 2>&1; rc=$?
tail -3 gpurun_out/t9_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/t9_tests.log | head -30; exit $rc; }
for v in dev host; do
  if [ $v = host ]; then export HZ_HOST_CODEBOOK=1 HZ_HOST_HEADER=1; fi
  timeout -k 10 300 python -u tools/cli_timing.py --gib 1 --out gpurun_out/cli1g_$v.json > gpurun_out/t9_cli_$v.log 2>&1 || { tail gpurun_out/t9_cli_$v.log; exit 6; }
  python -c "import json;d=json.load(open('gpurun_out/cli1g_$v.json'));print('$v', {k:(d[k]['host_ms'],d[k]['kernel_ms'],d[k]['total_ms']) for k in ('archive','extract')})"
done
