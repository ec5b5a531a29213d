#!/bin/bash
# Per-kernel averages (rocprofv3 kernel trace) of the index-less extract (tools/debug/extract_loop.py) under
# library variants (HZ_LIB_VARIANT dirs; "lib" = the product build), plus the timed loop's own numbers.
# usage (on the box): bash tools/exp_extract.sh SIZE REPS DIST dir1 dir2 ...
set -o pipefail
N=$1; R=$2; DIST=$3; shift 3
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in "$@"; do
  HZ_LIB_VARIANT=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/kx_$d -o run --output-format csv -- \
    python3 tools/debug/extract_loop.py $N $R $DIST --only-indexless > gpurun_out/kx_$d.log 2>&1 || { echo "variant $d failed"; tail -5 gpurun_out/kx_$d.log; exit 3; }
  grep "^rep" gpurun_out/kx_$d.log | tail -2
  f=$(find gpurun_out/kx_$d -name "run_kernel_stats.csv" | head -1)
  python3 - "$f" "$d" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "chain" in r["Name"] or "k_decode" in r["Name"] or "pack_write" in r["Name"]:
        print(sys.argv[2], r["Name"][:50], "calls", r["Calls"], "avg_ms %.3f" % (float(r["AverageNs"]) / 1e6))
PY
done
