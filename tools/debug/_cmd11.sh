set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in lib lib_ntl lib lib_ntl; do
  HZ_LIB_VARIANT=$v timeout -k 10 200 python tools/debug/stage_loop.py 17179869184 4 zipf p > gpurun_out/ploop_$v.log 2>&1 || { tail -5 gpurun_out/ploop_$v.log; exit 5; }
  echo "$v: $(grep -E 'rep (2|3)' gpurun_out/ploop_$v.log | grep -oE "'pack': [0-9.]+" | tr '\n' ' ')"
done
