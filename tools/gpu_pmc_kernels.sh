#!/bin/bash
# Per-KERNEL counters of one harness run (on the GPU box, repo root): HBM traffic (FETCH_SIZE and
# WRITE_SIZE in separate passes) and the SQ instruction / wait / LDS mix, one rocprofv3 pass per
# counter group, summarised per kernel by tools/pmc_kernels.py.
# usage: bash tools/gpu_pmc_kernels.sh TAG "harness command (python3 ...)"
#   e.g. bash tools/gpu_pmc_kernels.sh r05x "python3 tools/debug/extract_loop.py 17179869184 1 zipf --only-indexless"
set -o pipefail
T=$1; CMD=$2
O=gpurun_out/pmck_$T
mkdir -p $O
export TMPDIR=/tmp
GROUPS_=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH TA_TA_BUSY_sum TA_BUSY_avr"
)
i=0
for P in "${GROUPS_[@]}"; do
  i=$((i+1))
  # shellcheck disable=SC2086
  timeout -s KILL 240 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- $CMD > $O/p$i.log 2>&1 \
    || { echo "pass $i ($P) failed"; tail -5 $O/p$i.log; exit 3; }
done
python3 tools/pmc_kernels.py $O > $O/summary.txt && cat $O/summary.txt
