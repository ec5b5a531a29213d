set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in lib lib_dnt lib lib_dnt; do
  HZ_LIB_VARIANT=$v timeout -k 10 200 python tools/debug/stage_loop.py 17179869184 4 zipf d > gpurun_out/dloop_$v.log 2>&1 || { tail -5 gpurun_out/dloop_$v.log; exit 5; }
  echo "$v: $(grep -E 'rep (2|3)' gpurun_out/dloop_$v.log | grep -oE "'decode': [0-9.]+" | tr '\n' ' ')"
  HZ_LIB_VARIANT=$v timeout -k 10 200 python tools/debug/extract_loop.py 17179869184 2 zipf --only-indexless > gpurun_out/xl_$v.log 2>&1 || { tail -5 gpurun_out/xl_$v.log; exit 6; }
  echo "$v: $(grep rep gpurun_out/xl_$v.log | tr '\n' ' ')"
done
