# 16 GiB CLI stage split at 512 / 256 / 128 MiB extract windows
set -o pipefail
mkdir -p gpurun_out
for w in 536870912 268435456 134217728; do
  HZ_EXTRACT_WINDOW=$w timeout -k 10 600 python -u tools/cli_timing.py --gib 16 --out gpurun_out/cli16_w$w.json > gpurun_out/t11_$w.log 2>&1 || { tail gpurun_out/t11_$w.log; exit 6; }
  python -c "import json;d=json.load(open('gpurun_out/cli16_w$w.json'));print($w, {k:{x:d[k][x] for x in ('total_ms','fread_ms','fwrite_ms','alloc_ms','host_ms','kernel_ms','process_wall_s')} for k in ('archive','extract')}, d['round_trip_identical'])"
done
