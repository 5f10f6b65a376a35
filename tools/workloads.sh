#!/bin/bash
# Bench lines, one after the other, each under its own time limit:
#   tools/workloads.sh <tag> <name>[,<limit s>] ... 
# names: config2 pernode pernode_order config3 config3_order config4 config4pn config4pn_order dispatch
#        walk_spring walk_fall walk_after10d parse   (-> gpurun_out/<tag>/<name>.json)
set -o pipefail
O=gpurun_out/$1
shift
mkdir -p $O
declare -A A=(
  [config2]="--steps 20 --warmup 5"
  [pernode]="--workload pernode --steps 10 --warmup 2"
  [pernode_order]="--workload pernode --time-order --steps 10 --warmup 2"
  [config3]="--workload config3 --steps 2 --warmup 1"
  [config3_order]="--workload config3 --time-order --steps 2 --warmup 1"
  [config4]="--workload config4 --steps 4 --warmup 2"
  [config4pn]="--workload config4 --per-node --steps 2"
  [config4pn_order]="--workload config4 --per-node --time-order --steps 2"
  [dispatch]="--workload dispatch --steps 20 --warmup 3"
  [walk_spring]="--zone America/New_York --t0 1772910000 --steps 10 --warmup 3"
  [walk_fall]="--zone America/New_York --t0 1793469600 --steps 10 --warmup 3"
  [walk_after10d]="--zone America/New_York --t0 1773792000 --steps 10 --warmup 3"
  [parse]="--workload parse --steps 3 --warmup 1"
)
for spec in "$@"; do
  name=${spec%%,*}; lim=400
  [[ "$spec" == *,* ]] && lim=${spec#*,}
  [ -n "${A[$name]}" ] || { echo "unknown workload $name"; exit 2; }
  timeout -k 10 $lim python -u bench.py ${A[$name]} > $O/$name.json 2> $O/$name.err || { echo "FAILED $name"; tail -20 $O/$name.err; exit 1; }
  python3 tools/line.py $O/$name.json
done
