#!/bin/bash
# summary of a tools/gpu_check.sh run (local side)
T=$1
tail -1 gpurun_out/probe_$T.log 2>/dev/null; tail -n 1 gpurun_out/gpu_tests_$T.log 2>/dev/null
for f in gpurun_out/b_${T}_4g.json gpurun_out/b_${T}_zipf.json; do
  [ -f $f ] && python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['kernel_ms'],d['roundtrip_bit_exact'])"
done
