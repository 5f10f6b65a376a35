#!/bin/bash
# Writer time across separate bench processes on one box (allocation placement
# varies per process): tools/repeat_bench.sh <tag> <runs>
set -o pipefail
OUT=gpurun_out/${1:-repeat}
mkdir -p "$OUT"
for i in $(seq 1 ${2:-4}); do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > "$OUT/r$i.json" 2> "$OUT/r$i.err" \
    || { tail -20 "$OUT/r$i.err"; exit 1; }
  grep "times buffer" "$OUT/r$i.err"
  python3 -c "import json; d=json.load(open('$OUT/r$i.json')); print('run $i write_cf=%.4f ms step=%.4f ms' % (d['kernel_ms']['write_cf'], d['ms_per_step']))"
done
