#!/bin/bash
# Packed (offset, rule) merge: correctness (time-order GPU tests) and A/B (pernode / config3 --time-order)
set -o pipefail
O=gpurun_out/r4m9
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py -k "time or async or cmd_keys" > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/pytest.log | head; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for round in 1 2; do
for L in cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_pk5.so cronsun_amd/libcronsun_gpu_pk6.so cronsun_amd/libcronsun_gpu_nopk.so; do
  v=$(basename $L .so)
  CRONSUN_GPU_LIB=$L timeout -k 10 300 python -u bench.py --workload pernode --time-order --steps 10 --cpu-sample 0 --verify-sample 250 > $O/$v.$round.json 2> $O/$v.$round.err || { echo "fail $v"; tail -5 $O/$v.$round.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.$round.json')); print('$v', 'pernode-to ms/step %.3f' % d['ms_per_step'], 'node_write+order %.3f' % d['kernel_ms']['node_write'], d['verified'])"
done
done
for L in cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_pk6.so cronsun_amd/libcronsun_gpu_nopk.so; do
  v=$(basename $L .so)
  CRONSUN_GPU_LIB=$L timeout -k 10 300 python -u bench.py --workload config3 --time-order --steps 1 --warmup 1 --cpu-sample 0 --verify-sample 250 > $O/c3_$v.json 2> $O/c3_$v.err || { echo "fail c3 $v"; tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$v.json')); print('$v', 'config3-to ms/step %.1f' % d['ms_per_step'], d['verified'])"
done
