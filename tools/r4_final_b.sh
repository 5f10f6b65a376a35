#!/bin/bash
# Round-4 final (b): the other workloads' bench lines (CPU baselines included) -> gpurun_out/r4fb
set -o pipefail
O=gpurun_out/r4fb
mkdir -p $O
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); cb=d.get('cpu_baseline') or {}; print('$tag', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'], 'cpu %.3g' % (cb.get('value') or 0), d['verified'], (d.get('verify') or {}).get('every_step', {}).get('mismatches'))"
}
run pernode --workload pernode --steps 20
run pernode_to --workload pernode --time-order --steps 10
run config3 --workload config3 --steps 2 --warmup 1
run config3_to --workload config3 --time-order --steps 1 --warmup 1
run config4 --workload config4 --steps 3 --warmup 1
run dispatch --workload dispatch --steps 30
run ny_spring --zone America/New_York --t0 1772910000 --steps 20 --cpu-sample 0
