#!/bin/bash
# Secondary bench lines on the final tree: pernode, pernode --time-order, config3, config4, dispatch,
# and config 2 in America/New_York on both 2026 DST days and ten days after the spring-forward.
#   tools/final_workloads.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r3_fin}
mkdir -p $O
run() {  # name, seconds, bench args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "FAILED $name"; tail -20 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$name.json')); r=d.get('roofline') or {}; print('$name', '%.4g' % d['value'], d['unit'], 'ms/step %.3f' % d['ms_per_step'], 'frac', r.get('frac'), 'verified', d.get('verified'))"
}
run pernode 300 --workload pernode --steps 10 --warmup 2
run pernode_order 300 --workload pernode --time-order --steps 6 --warmup 2
run config4 400 --workload config4 --steps 4 --warmup 2
run dispatch 300 --workload dispatch --steps 20 --warmup 3
run walk_spring 300 --zone America/New_York --t0 1772910000 --steps 10 --warmup 3
run walk_fall 300 --zone America/New_York --t0 1793469600 --steps 10 --warmup 3
run walk_after10d 300 --zone America/New_York --t0 1773792000 --steps 10 --warmup 3
run config3 400 --workload config3 --steps 2 --warmup 1
