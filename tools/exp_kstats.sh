#!/bin/bash
# Per-kernel averages (rocprofv3 kernel trace) of one stage of tools/debug/stage_loop.py under library variants.
# usage (on the box): bash tools/exp_kstats.sh STAGES SIZE DIST KERNEL_REGEX dir1 dir2 ...
set -o pipefail
ST=$1; SIZE=$2; DIST=$3; RX=$4; shift 4
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in "$@"; do
  HZ_LIB_VARIANT=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ks_$d -o run --output-format csv -- \
    python3 tools/debug/stage_loop.py $SIZE 3 $DIST $ST > gpurun_out/ks_$d.log 2>&1 || { echo "variant $d failed"; tail -5 gpurun_out/ks_$d.log; exit 3; }
  f=$(find gpurun_out/ks_$d -name "run_kernel_stats.csv" | head -1)
  python3 - "$f" "$RX" "$d" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r["Name"]):
        print(sys.argv[3], r["Name"][:60], "calls", r["Calls"], "avg_ms %.3f" % (float(r["AverageNs"]) / 1e6))
PY
done
