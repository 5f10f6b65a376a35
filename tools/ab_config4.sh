#!/bin/bash
# A/B of library variants (built with make OUT=../libcronsun_gpu_<suffix>.so):
#   WL=config4 tools/ab_config4.sh <tag> <lib-suffix|base>...   (WL default config4)
# Two interleaved rounds, so box drift shows as a spread, not as a difference.
set -o pipefail
OUT=gpurun_out/${1:-ab4}
shift
WL=${WL:-config4}
STEPS=${STEPS:-3}
mkdir -p "$OUT"
for round in 1 2; do
for v in "$@"; do
  [ "$v" = base ] && v=""
  f="$OUT/${WL}_${v:-base}_$round"
  CRONSUN_GPU_LIB=$PWD/cronsun_amd/libcronsun_gpu${v:+_$v}.so timeout -k 10 400 python bench.py --workload $WL \
    --steps $STEPS --warmup 1 --cpu-sample 0 --verify-sample 200 > "$f.json" 2> "$f.err" || { tail -20 "$f.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$f.json')); k=d['kernel_ms']; print('%-8s %s round $round count=%.4f scan=%.4f write_cf=%.3f node_write=%s segs=%s step=%.4f ms verified=%s' % ('${v:-base}', '$WL', k['count'], k['scan'], k['write_cf'], k.get('node_write'), k.get('segments_and_offsets'), d['ms_per_step'], d['verified']))"
done
done
