# PMC passes over one stage of tools/debug/stage_loop.py (4 GiB Zipf): instruction mix, waits, LDS and TA
# usage: bash tools/gpu_pmc_stage.sh STAGE(h|p|d|i) OUTDIR
set -o pipefail
ST=${1:-d}; O=${2:-gpurun_out/pmc_$ST}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH TA_TA_BUSY_sum TA_BUSY_avr TD_TD_BUSY_sum GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- python3 tools/debug/stage_loop.py 4294967296 2 zipf $ST > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 5; }
done
python3 - "$O" <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/p*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    if any(x in k for x in ("decode", "pack_write", "pack_count", "hist16", "idx_walk", "sync_select")):
        print(k, {c: f"{v:.3e}" for c, v in sorted(d.items())})
PY
