# PMC: k_seg_walk with and without piece records (4 GiB Zipf)
set -o pipefail
O=gpurun_out/pmc9
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_COUNT"
for v in lib lib_norec; do
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  HZ_LIB_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $P -d $O/${v}_$i -o run --output-format csv -- python3 tools/debug/extract_loop.py 4294967296 1 zipf --only-indexless > $O/${v}_$i.log 2>&1 || { tail -5 $O/${v}_$i.log; exit 5; }
done
done
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w -o run --output-format csv -- python3 tools/debug/extract_loop.py 4294967296 1 zipf --only-indexless > $O/w.log 2>&1 || { tail -5 $O/w.log; exit 6; }
python3 - "$O" <<'PY'
import csv, glob, collections, sys, os
for sub in ["lib", "lib_norec", "w"]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(sys.argv[1] + "/" + sub + "*/**/run_counter_collection.csv", recursive=True):
        if sub == "lib" and "norec" in f: continue
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-16:]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in acc.items():
        if "seg_walk" in k or "piece" in k:
            print(sub, k, {c: f"{v:.3e}" for c, v in sorted(d.items())})
PY
