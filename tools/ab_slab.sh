#!/bin/bash
# Slab writer A/B on one box: tools/ab_slab.sh <tag> <bench args...>; libraries
# from $LIBS (paths under cronsun_amd/), each with CG_ORDER_SLAB=1, then the
# default library with CG_ORDER_SLAB=0 (tile sort + merge)
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
for L in $LIBS; do
  v=$(basename $L .so)
  CG_ORDER_SLAB=1 CRONSUN_GPU_LIB=$L timeout -k 10 300 python -u bench.py "$@" --cpu-sample 0 --verify-sample 0 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 tools/line.py $O/$v.json | head -2
done
CG_ORDER_SLAB=0 timeout -k 10 300 python -u bench.py "$@" --cpu-sample 0 --verify-sample 0 > $O/tiles.json 2> $O/tiles.err || exit 1
python3 tools/line.py $O/tiles.json | head -2
