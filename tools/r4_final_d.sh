#!/bin/bash
# Round-4 final (d), after the packed time-order words: the GPU suite + smoke + headline + its rocprof
# stats and PMC (r4_final_a into gpurun_out/r4fd), then the two time-order bench lines with CPU baselines
set -o pipefail
sed 's#O=gpurun_out/r4fa#O=gpurun_out/r4fd#; s#r4fa/suite#r4fd/suite#' tools/r4_final_a.sh > /tmp/r4_final_d_a.sh
bash /tmp/r4_final_d_a.sh || exit 1
O=gpurun_out/r4fd
for w in pernode_to config3_to; do
  case $w in
    pernode_to) args="--workload pernode --time-order --steps 10";;
    config3_to) args="--workload config3 --time-order --steps 1 --warmup 1";;
  esac
  timeout -k 10 400 python -u bench.py $args > $O/$w.json 2> $O/$w.err || { echo "bench $w failed"; tail -20 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('$w', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'], d['verified'], d['verify']['every_step']['mismatches'])"
done
