#!/bin/bash
# Interleaved comparison of several in-tree builds on one bench line:
#   tools/ab_libs.sh <tag> "<lib1> <lib2> ..." <bench args...>
# (each lib a path under cronsun_amd/; two rounds, interleaved)
set -o pipefail
O=gpurun_out/$1; LIBS=$2; shift 2
mkdir -p $O
for round in 1 2; do
  for L in $LIBS; do
    v=$(basename $L .so)
    CRONSUN_GPU_LIB=$L timeout -k 10 300 python -u bench.py "$@" --cpu-sample 0 --verify-sample 250 > $O/$v.$round.json 2> $O/$v.$round.err || { tail -5 $O/$v.$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$round.json')); k=d['kernel_ms']; print('$v', 'step %.3f' % d['ms_per_step'], {a: round(b, 3) for a, b in k.items() if isinstance(b, float) and b > 0.05}, d['verified'])" | tee -a $O/summary.txt
  done
done
