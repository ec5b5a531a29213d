# PMC passes (instruction mix, waits, LDS, TA) for the extract kernels and k_decode, 4 GiB Zipf
set -o pipefail
O=gpurun_out/pmc7
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH TA_TA_BUSY_sum TA_BUSY_avr TD_TD_BUSY_sum GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/x$i -o run --output-format csv -- python3 tools/debug/extract_loop.py 4294967296 1 zipf --only-indexless > $O/x$i.log 2>&1 || { tail -5 $O/x$i.log; exit 5; }
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/d$i -o run --output-format csv -- python3 tools/debug/stage_loop.py 4294967296 1 zipf d > $O/d$i.log 2>&1 || { tail -5 $O/d$i.log; exit 6; }
done
python3 - "$O" <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-30:]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    if any(x in k for x in ("piece_decode", "seg_walk", "k_decode<")):
        print(k, {c: f"{v:.3e}" for c, v in sorted(d.items())})
PY
