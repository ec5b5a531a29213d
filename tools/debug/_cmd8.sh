set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in lib lib_hd16 lib_hd4 lib lib_hd16; do
  HZ_LIB_VARIANT=$v timeout -k 10 200 python tools/debug/stage_loop.py 17179869184 4 zipf h > gpurun_out/hloop_$v.log 2>&1 || { tail -5 gpurun_out/hloop_$v.log; exit 5; }
  echo "$v: $(grep -E 'rep (2|3)' gpurun_out/hloop_$v.log | cut -c1-60 | tr '\n' ' ')"
done
