#!/bin/bash
# Per-kernel times of the index build under library variants (rocprofv3 kernel stats).
# usage (on the box): bash tools/exp_walk_prof.sh SIZE REPS dir1 dir2 ...
set -o pipefail
N=$1; shift; R=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  HZ_LIB_VARIANT=$v timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/ewp_$v -o run --output-format csv -- \
    python3 tools/debug/index_ab.py $N $R > gpurun_out/ewp_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/ewp_$v.log; exit 3; }
  grep "index ms" gpurun_out/ewp_$v.log
  python3 - gpurun_out/ewp_$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(k in n for k in ("k_idx", "k_sync", "k_scan")):
        print("   %-40s %4s %9.3f ms" % (n.split("(")[0][:40], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
done
