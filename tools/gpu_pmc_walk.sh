# PMC passes over the index build (4 GiB Zipf): instruction mix and wait share of k_idx_walk / k_sync_select
set -o pipefail
mkdir -p gpurun_out/pmcw
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/pmcw/p$i -o run --output-format csv -- python3 tools/debug/stage_loop.py 4294967296 2 zipf i > gpurun_out/pmcw/p$i.log 2>&1 || { tail -5 gpurun_out/pmcw/p$i.log; exit 5; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/pmcw/p*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-30:]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    if "walk" in k or "select" in k:
        print(k, {c: f"{v:.3e}" for c, v in sorted(d.items())})
PY
