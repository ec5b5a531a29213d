# bench.py under library variants (HZ_LIB_VARIANT dirs; "lib" = the product build), alternating:
# prints per run ms/step and the stage kernel times (a run that is not bit-exact still prints, ok False).  usage: bash tools/debug/bench_ab.sh REPS dir1 dir2 ...
set -o pipefail
R=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for v in "$@"; do
    HZ_LIB_VARIANT=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bab_$v.json 2> gpurun_out/bab_$v.err \
      || { [ -s gpurun_out/bab_$v.json ] || { echo "variant $v failed"; tail -5 gpurun_out/bab_$v.err; exit 3; }; }
    python3 -c "
import json,sys; j=json.loads(open('gpurun_out/bab_$v.json').read().strip().splitlines()[-1])
print('%-10s %8.3f ms/step %8.2f GB/s  kernels %s  dropin %.3f ms (extract %.3f)  ok %s' % ('$v', j['ms_per_step'], j['value'], j['kernel_ms'], j['dropin']['ms_per_step'], j['dropin']['kernel_ms'].get('extract', 0), j['roundtrip_bit_exact']))"
  done
done
