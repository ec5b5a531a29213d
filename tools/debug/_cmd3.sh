set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/xprof -o xprof -- python3 tools/debug/extract_loop.py 17179869184 2 zipf --only-indexless > gpurun_out/xprof.log 2>&1 || { tail -20 gpurun_out/xprof.log; exit 2; }
grep rep gpurun_out/xprof.log
f=$(find gpurun_out/xprof -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -25
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sprof -o sprof -- python3 tools/debug/stage_loop.py 17179869184 3 zipf hpd > gpurun_out/sprof.log 2>&1 || { tail -20 gpurun_out/sprof.log; exit 3; }
f=$(find gpurun_out/sprof -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -25
