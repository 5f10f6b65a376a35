#!/bin/bash
# A/B of library builds over expansion horizons (config-2 mix, 1M rules) and
# the pernode workload: tools/ab_horizon.sh <tag> <lib-suffix|base>...
set -o pipefail
OUT=gpurun_out/${1:-abh}
shift
mkdir -p "$OUT"
for v in "$@"; do
  [ "$v" = base ] && v=""
  lib=$PWD/cronsun_amd/libcronsun_gpu${v:+_$v}.so
  for h in 60 3600 86400; do
    f="$OUT/${v:-base}_h$h"
    CRONSUN_GPU_LIB=$lib timeout -k 10 200 python bench.py --horizon $h --steps 20 --warmup 3 --cpu-sample 0 \
      --verify-sample 500 > "$f.json" 2> "$f.err" || { tail -20 "$f.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$f.json')); print('%-6s h=%-6d E=%-10d write=%.4f step=%.4f ms verified=%s' % ('${v:-base}', $h, d['config']['events_per_gpu_step'], d['kernel_ms']['write_cf'], d['ms_per_step'], d['verified']))"
  done
  f="$OUT/${v:-base}_pernode"
  CRONSUN_GPU_LIB=$lib timeout -k 10 300 python bench.py --workload pernode --steps 5 --warmup 2 --cpu-sample 0 \
    > "$f.json" 2> "$f.err" || { tail -20 "$f.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$f.json')); k=d['kernel_ms']; print('%-6s pernode write=%.4f node_write=%.4f step=%.4f ms verified=%s' % ('${v:-base}', k['write_cf'], k['node_write'], d['ms_per_step'], d['verified']))"
done
