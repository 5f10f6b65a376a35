#!/bin/bash
# GPU suite + smoke + headline, then k_node_write blocks-per-CU A/B on pernode
set -o pipefail
bash tools/r4_gpu_suite.sh r4_suite1 || exit 1
O=gpurun_out/r4m3
mkdir -p $O
for round in 1 2; do
for L in cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_nb2.so cronsun_amd/libcronsun_gpu_nb3.so cronsun_amd/libcronsun_gpu_nb4.so; do
  v=$(basename $L .so)
  CRONSUN_GPU_LIB=$L timeout -k 10 300 python -u bench.py --workload pernode --steps 10 --cpu-sample 0 --verify-sample 0 > $O/$v.$round.json 2> $O/$v.$round.err || { echo "fail $v"; tail -5 $O/$v.$round.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.$round.json')); print('$v', 'ms/step %.3f' % d['ms_per_step'], 'node_write %.3f' % d['kernel_ms']['node_write'])"
done
done
