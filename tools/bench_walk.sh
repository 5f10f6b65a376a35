#!/bin/bash
# Walk-path bench: config 2 (1M rules x 24 h) in America/New_York on the 24 h
# around the 2026 DST transitions (spring-forward 2026-03-08 07:00Z, fall-back
# 2026-11-01 06:00Z) and on 2026-03-18 (ten days after the spring-forward), plus a kernel trace of each (k_count / k_write_cf /
# k_write_walk).   tools/bench_walk.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-walk}
mkdir -p "$OUT"
export TMPDIR=/tmp
for day in spring:1772910000 fall:1793469600 after10d:1773792000; do
  name=${day%%:*}
  t0=${day##*:}
  B="bench.py --zone America/New_York --t0 $t0 --steps 10 --warmup 3"
  timeout -k 10 400 python -u $B > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); k=d['kernel_ms']; print('$name', '%.4g ev/s' % d['value'], 'step %.3f ms' % d['ms_per_step'], 'count %.4f write_cf %.4f walk %.4f' % (k['count'], k['write_cf'], k['write_walk']), 'frac %.3f' % d['roofline']['frac'], 'verified', d['verified'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -- \
    python3 $B --cpu-sample 0 --verify-sample 0 > "$OUT/${name}_prof.json" 2> "$OUT/prof_$name.err" \
    || { tail -20 "$OUT/prof_$name.err"; exit 1; }
  find "$OUT/prof_$name" -name '*kernel_stats.csv' -exec cat {} \;
done
