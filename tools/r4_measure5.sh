#!/bin/bash
# Writer layout A/B (config 2) and time-order merge A/B (pernode, config3)
set -o pipefail
bash tools/ab_libs.sh r4m5/ab "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_s10.so cronsun_amd/libcronsun_gpu_pl.so cronsun_amd/libcronsun_gpu_w2.so cronsun_amd/libcronsun_gpu_w8.so" --steps 30 --warmup 5 || exit 1
O=gpurun_out/r4m5/order
mkdir -p $O
for round in 1 2; do
for L in cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_mw8.so cronsun_amd/libcronsun_gpu_os.so cronsun_amd/libcronsun_gpu_osmw8.so; do
  v=$(basename $L .so)
  CRONSUN_GPU_LIB=$L timeout -k 10 300 python -u bench.py --workload pernode --time-order --steps 10 --cpu-sample 0 --verify-sample 250 > $O/$v.$round.json 2> $O/$v.$round.err || { echo "fail $v"; tail -5 $O/$v.$round.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.$round.json')); print('$v', 'pernode-to ms/step %.3f' % d['ms_per_step'], 'node_write+order %.3f' % d['kernel_ms']['node_write'], d['verified'])"
done
done
for L in cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_mw8.so cronsun_amd/libcronsun_gpu_osmw8.so; do
  v=$(basename $L .so)
  CRONSUN_GPU_LIB=$L timeout -k 10 300 python -u bench.py --workload config3 --time-order --steps 1 --warmup 1 --cpu-sample 0 --verify-sample 250 > $O/c3_$v.json 2> $O/c3_$v.err || { echo "fail c3 $v"; tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$v.json')); print('$v', 'config3-to ms/step %.1f' % d['ms_per_step'], d['verified'])"
done
