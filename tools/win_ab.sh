#!/bin/bash
# config 4 per node at several window lengths (one box): tools/win_ab.sh <tag> <seconds>...
O=gpurun_out/$1; shift; mkdir -p $O
for w in "$@"; do
  timeout -k 10 400 python -u bench.py --workload config4 --per-node --window $w --steps 2 --warmup 1 --cpu-sample 0 --verify-sample 250 > $O/w$w.json 2> $O/w$w.err
  rc=$?
  case $rc in 0) python3 tools/line.py $O/w$w.json ;; 124|134|137|139) echo "w$w rc $rc: stop"; exit $rc ;; *) echo "w$w rc $rc"; tail -3 $O/w$w.err ;; esac
done
