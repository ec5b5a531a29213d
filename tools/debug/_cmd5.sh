set -o pipefail
mkdir -p gpurun_out/pmcx
export TMPDIR=/tmp
for v in lib lib_nt0; do
 for c in WRITE_SIZE FETCH_SIZE; do
  HZ_LIB_VARIANT=$v timeout -k 10 240 rocprofv3 --pmc $c -d gpurun_out/pmcx/${v}_$c -o run --output-format csv -- python3 tools/debug/extract_loop.py 17179869184 1 zipf --only-indexless > gpurun_out/pmcx/${v}_$c.log 2>&1 || { tail -5 gpurun_out/pmcx/${v}_$c.log; exit 3; }
 done
done
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob('gpurun_out/pmcx/*/**/*counter_collection.csv', recursive=True)):
    agg = {}
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:40]
        if 'seg' in k or 'scan' in k:
            agg[(k, r['Counter_Name'])] = agg.get((k, r['Counter_Name']), 0.0) + float(r['Counter_Value'])
    print(f.split('/')[2], {f'{k[0]}:{k[1]}': round(v / 1e6, 3) for k, v in agg.items()}, '(GB, KiB units x1e-6)')
PY
