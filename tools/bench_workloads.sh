#!/bin/bash
# Secondary bench workloads on the current tree: tools/bench_workloads.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-wl}
mkdir -p "$OUT"
for wl in pernode config4 dispatch; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 5 --warmup 2 > "$OUT/$wl.json" 2> "$OUT/$wl.err" \
    || { tail -20 "$OUT/$wl.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$wl.json')); print('$wl', '%.4g' % d['value'], d['unit'], 'ms/step %.3f' % d['ms_per_step'])"
done
