#!/bin/bash
# A/B of library variants on config 4 (10M x 7 d): tools/ab_config4.sh <tag> <lib-suffix>...
set -o pipefail
OUT=gpurun_out/${1:-ab4}
shift
mkdir -p "$OUT"
for v in "$@"; do
  [ "$v" = base ] && v=""
  CRONSUN_GPU_LIB=$PWD/cronsun_amd/libcronsun_gpu${v:+_$v}.so timeout -k 10 400 python bench.py --workload config4 \
    --steps 3 --warmup 1 --cpu-sample 0 > "$OUT/${v:-base}.json" 2> "$OUT/${v:-base}.err" || { tail -20 "$OUT/${v:-base}.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/${v:-base}.json')); print('%-8s config4 write_cf=%.3f ms step=%.3f ms' % ('${v:-base}', d['kernel_ms']['write_cf'], d['ms_per_step']))"
done
