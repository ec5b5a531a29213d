#!/bin/bash
# Profiling recipe for one round (run on the GPU box from the repo root):
#   gpurun -- 'bash tools/profile_round.sh r01'
# 1. rocprofv3 kernel-trace stats of the default bench command (Zipf and uniform)
# 2. separate FETCH_SIZE / WRITE_SIZE counter passes (never combined with traces)
#    -> gpurun_out/pmc_traffic.json (tools/pmc_traffic.py applies the gfx950 corrections)
# 3. PMC calibration of the access shapes the kernels use (tools/microbench/mb_pmc_calib.hip)
# 4. the default bench line (Zipf, CPU baseline) with the measured traffic
set -e -o pipefail
R=${1:-r01}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
for D in zipf uniform; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats_$D -o run --output-format csv -- \
    python3 bench.py --dist $D --steps 5 --warmup 2 --no-cpu-baseline > $O/stats_$D.log 2>&1
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$D -o run --output-format csv -- \
    python3 bench.py --dist $D --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch_$D.log 2>&1
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/write_$D -o run --output-format csv -- \
    python3 bench.py --dist $D --steps 1 --warmup 0 --no-cpu-baseline > $O/write_$D.log 2>&1
  python3 tools/pmc_traffic.py --fetch $O/fetch_$D --write $O/write_$D --dist $D --size $((16 << 30)) \
    --out $O/pmc_traffic.json
  # the extract path alone (its count scans share kernel names with the index builder's)
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/xfetch_$D -o run --output-format csv -- \
    python3 tools/debug/extract_loop.py $((16 << 30)) 1 $D --only-indexless > $O/xfetch_$D.log 2>&1
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/xwrite_$D -o run --output-format csv -- \
    python3 tools/debug/extract_loop.py $((16 << 30)) 1 $D --only-indexless > $O/xwrite_$D.log 2>&1
  python3 tools/pmc_traffic.py --fetch $O/xfetch_$D --write $O/xwrite_$D --dist $D --size $((16 << 30)) \
    --out $O/pmc_traffic.json
done
if [ -x tools/microbench/mbc ]; then
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch -o run --output-format csv -- \
    tools/microbench/mbc > $O/calib_fetch.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $O/calib_write -o run --output-format csv -- \
    tools/microbench/mbc > $O/calib_write.log 2>&1
fi
timeout -k 10 600 python3 bench.py --profile-json $O/pmc_traffic.json > $O/bench_zipf.json 2> $O/bench_zipf.err
timeout -k 10 300 python3 bench.py --dist uniform --profile-json $O/pmc_traffic.json > $O/bench_uniform.json 2> $O/bench_uniform.err
