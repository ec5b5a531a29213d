set -o pipefail
mkdir -p gpurun_out/r02i
export TMPDIR=/tmp
HZ_IDX_SEG=512 timeout -k 10 120 python tools/debug/index_diff.py 1 6291457 > gpurun_out/r02i/diff.log 2>&1 || exit 1
HZ_IDX_SEG=256 timeout -k 10 120 python tools/debug/index_diff.py 1 1048576 >> gpurun_out/r02i/diff.log 2>&1 || exit 1
for cfg in "0 512" "0 1024" "0 2048" "2 512"; do
  set -- $cfg
  HZ_IDX_WALK=$1 HZ_IDX_SEG=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02i/prof_$1_$2 -o run --output-format csv -- python3 tools/debug/stage_loop.py 4294967296 2 zipf i > gpurun_out/r02i/prof_$1_$2.log 2>&1 || exit 2
done
