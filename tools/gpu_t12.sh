# index build timing: product vs the no-escape-gather experiment (wrong lengths; timing only)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for d in lib lib_noesc; do
  HZ_LIB_VARIANT=$d timeout -k 10 120 python tools/debug/stage_loop.py 17179869184 3 zipf i > gpurun_out/t12_${d}_$r.log 2>&1 || { echo "$d failed"; tail -3 gpurun_out/t12_${d}_$r.log; }
  echo "$d r$r: $(grep '^rep 2' gpurun_out/t12_${d}_$r.log)"
done
done
