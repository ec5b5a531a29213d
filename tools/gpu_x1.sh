# Development GPU check of the index-less extract (on the box, repo root): its tests, the split-over-ranks
# rehearsal, then rocprofv3 kernel stats of the 16 GiB Zipf extract (tools/debug/extract_loop.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_dist.py -k "indexless" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/x1.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/x1.log | tail -40; [ $rc -eq 0 ] || HZ_CAPTURE_DEBUG=1 timeout -k 10 100 python3 tools/debug/x_capture.py global 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/x1prof -o run --output-format csv -- python3 tools/debug/extract_loop.py 17179869184 3 zipf > gpurun_out/x1loop.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/x1loop.log; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/x1prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-50s %5s %9.3f ms" % (r["Name"].split("(")[0][:50], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
