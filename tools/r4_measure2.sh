#!/bin/bash
# A/B of the per-node paths across builds (round-3 16-B records + tile pass,
# fused tile, fused tile + 8-B records) and kernel traces of the time order.
set -o pipefail
O=gpurun_out/r4m2
mkdir -p $O
export TMPDIR=/tmp
for round in 1 2; do
for L in cronsun_amd/libcronsun_gpu_d7c4dcb.so cronsun_amd/libcronsun_gpu_f9e2583.so cronsun_amd/libcronsun_gpu.so; do
  for w in "pernode" "pernode --time-order"; do
    v=$(basename $L .so); tag=$(echo $w | tr ' ' '_' | tr -d '-')
    CRONSUN_GPU_LIB=$L timeout -k 10 300 python -u bench.py --workload $w --steps 10 --cpu-sample 0 --verify-sample 0 > $O/$v.$tag.$round.json 2> $O/$v.$tag.$round.err || { echo "fail $v $w"; tail -5 $O/$v.$tag.$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$tag.$round.json')); print('$v', '$w', 'ms/step %.3f' % d['ms_per_step'], 'node_write %.3f' % d['kernel_ms']['node_write'])"
  done
done
done
for L in cronsun_amd/libcronsun_gpu_d7c4dcb.so cronsun_amd/libcronsun_gpu.so; do
  v=$(basename $L .so)
  CRONSUN_GPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -- python3 bench.py --workload pernode --time-order --steps 5 --cpu-sample 0 --verify-sample 0 > $O/prof_$v.json 2> $O/prof_$v.err || { echo "prof fail $v"; tail -5 $O/prof_$v.err; exit 1; }
  echo "== $v"; find $O/prof_$v -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-4 | head -30
done
