#!/bin/bash
# A/B of k_write_cf build variants on the bench workload (same box, interleaved):
#   tools/ab_write.sh <tag> <lib-suffix>...   (suffix "" = the default build)
set -o pipefail
OUT=gpurun_out/${1:-ab}
shift
mkdir -p "$OUT"
for round in 1 2; do
  for v in "$@"; do
    [ "$v" = base ] && v=""
    lib=$PWD/cronsun_amd/libcronsun_gpu${v:+_$v}.so
    CRONSUN_GPU_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 0 \
      > "$OUT/${v:-base}_$round.json" 2> "$OUT/${v:-base}_$round.err" || { tail -20 "$OUT/${v:-base}_$round.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v:-base}_$round.json')); print('%-8s r$round count=%.4f write_cf=%.4f ms step=%.4f ms' % ('${v:-base}', d['kernel_ms']['count'], d['kernel_ms']['write_cf'], d['ms_per_step']))"
  done
done
