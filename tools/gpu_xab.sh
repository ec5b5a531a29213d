# Index-less extract A/B on the GPU box: rocprofv3 kernel stats of tools/debug/extract_loop.py (16 GiB Zipf,
# --only-indexless) under each library variant (HZ_LIB_VARIANT dirs; "lib" = the product build).
# usage: bash tools/gpu_xab.sh SIZE REPS dir1 dir2 ...   (XAB_FULL=1: also index build + k_decode each rep)
set -o pipefail
N=$1; shift; R=$1; shift
ONLY=--only-indexless; [ -n "$XAB_FULL" ] && ONLY=
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  HZ_LIB_VARIANT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/xab_$v -o run --output-format csv -- \
    python3 tools/debug/extract_loop.py $N $R zipf $ONLY > gpurun_out/xab_$v.log 2>&1 \
    || { echo "variant $v failed"; tail -5 gpurun_out/xab_$v.log; exit 3; }
  echo "== $v: $(grep '^rep' gpurun_out/xab_$v.log | tr '\n' ' ')"
  python3 - gpurun_out/xab_$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(k in n for k in ("k_chain", "k_scan", "k_decode")):
        print("   %-40s %4s %9.3f ms" % (n.split("(")[0][:40], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
done
