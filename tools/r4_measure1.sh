#!/bin/bash
# Round 4 measurements: comm test (exit clean), writer occupancy A/B on config 2,
# pernode / pernode --time-order / config3 --time-order bench lines.
set -o pipefail
O=gpurun_out/r4m1
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_comm.py > $O/comm.log 2>&1 || { echo "comm failed rc $?"; tail -5 $O/comm.log; exit 1; }
tail -1 $O/comm.log
bash tools/ab_libs.sh r4m1/ab "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_np3.so cronsun_amd/libcronsun_gpu_np2.so cronsun_amd/libcronsun_gpu_np3s12.so" --steps 30 --warmup 5 || exit 1
for w in "pernode" "pernode --time-order" "config3 --time-order --steps 2 --warmup 1"; do
  tag=$(echo $w | tr ' ' '_' | tr -d '-')
  timeout -k 10 400 python -u bench.py --workload $w > $O/$tag.json 2> $O/$tag.err || { echo "bench $w failed"; tail -20 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$w', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['kernel_ms'].items() if not isinstance(v, str)}, d['verified'], d['verify'].get('every_step', {}).get('mismatches'))"
done
