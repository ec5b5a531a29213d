set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in lib; do
  HZ_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/x6_$v -o x --output-format csv -- python3 tools/debug/extract_loop.py 17179869184 2 zipf --only-indexless > gpurun_out/x6_$v.log 2>&1 || { tail -20 gpurun_out/x6_$v.log; exit 5; }
  f=$(find gpurun_out/x6_$v -name '*kernel_stats.csv' | head -1); echo "$v: $(grep -E 'k_seg_walk|k_piece_decode' $f | cut -d, -f1,4 | tr '\n' ' ')"
done
