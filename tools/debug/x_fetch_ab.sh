# FETCH_SIZE / WRITE_SIZE of the index-less extract's kernels under library variants (HZ_LIB_VARIANT dirs).
# usage: bash tools/debug/x_fetch_ab.sh SIZE dir1 dir2 ...
set -o pipefail
N=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    HZ_LIB_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/xf_${v}_$C -o run --output-format csv -- \
      python3 tools/debug/extract_loop.py $N 1 zipf --only-indexless > gpurun_out/xf_${v}_$C.log 2>&1 \
      || { echo "variant $v $C failed"; tail -5 gpurun_out/xf_${v}_$C.log; exit 3; }
    python3 - gpurun_out/xf_${v}_$C $C $v <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
t = defaultdict(float); n = defaultdict(int)
for r in csv.DictReader(open(f)):
    if r["Counter_Name"] != sys.argv[2] or "k_chain" not in r["Kernel_Name"]:
        continue
    k = r["Kernel_Name"].split("(")[0].split("::")[-1]
    t[k] += float(r["Counter_Value"]) * 1024; n[k] += 1
for k in sorted(t):
    print("%-10s %-10s %-24s %8.3f GB raw per launch" % (sys.argv[3], sys.argv[2], k, t[k] / n[k] / 1e9))
PY
  done
done
