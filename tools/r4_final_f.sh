#!/bin/bash
# Round-4 final (f): the GPU suite + smoke + headline on the final tree, then the time-order bench lines
set -o pipefail
bash tools/r4_gpu_suite.sh r4ff/suite || exit 1
O=gpurun_out/r4ff
for w in pernode_to config3_to; do
  case $w in
    pernode_to) args="--workload pernode --time-order --steps 10";;
    config3_to) args="--workload config3 --time-order --steps 1 --warmup 1";;
  esac
  timeout -k 10 400 python -u bench.py $args > $O/$w.json 2> $O/$w.err || { echo "bench $w failed"; tail -20 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('$w', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'], d['verified'], d['verify']['every_step']['mismatches'])"
done
