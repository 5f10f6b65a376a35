#!/bin/bash
# config 3 (rule order) at several window lengths (one box, two rounds): tools/win_ab_c3.sh <tag> <seconds>...
O=gpurun_out/$1; shift; mkdir -p $O
for round in 1 2; do
  for w in "$@"; do
    timeout -k 10 300 python -u bench.py --workload config3 --window $w --steps 2 --warmup 1 --cpu-sample 0 --verify-sample 250 > $O/w$w.$round.json 2> $O/w$w.$round.err
    rc=$?
    case $rc in 0) python3 tools/line.py $O/w$w.$round.json | cut -c1-120 ;; 124|134|137|139) echo "w$w rc $rc: stop"; exit $rc ;; *) echo "w$w rc $rc"; tail -3 $O/w$w.$round.err ;; esac
  done
done
