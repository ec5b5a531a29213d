set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/x1.log 2>&1
rc=$?; tail -25 gpurun_out/x1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/x1prof -o run --output-format csv -- python3 tools/debug/extract_loop.py 17179869184 3 zipf > gpurun_out/x1loop.log 2>&1
rc=$?; cat gpurun_out/x1loop.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/x1prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-50s %5s %9.3f ms" % (r["Name"].split("(")[0][:50], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
