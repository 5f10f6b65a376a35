#!/bin/bash
# merge split by node density, dense nodes (8-wave merge) on their own stream: parity, then A/B against dn0 (every node 4-wave) and dn4k (threshold 4096)
# merge split by node density, dense nodes (8-wave merge) on their own stream: parity, then A/B against dn0 (every node 4-wave) and dn4k (threshold 4096)
set -o pipefail
O=gpurun_out/r4m17
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py tests/test_gpu_config3_day.py -k "time or order or config3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/ab_libs.sh r4m17/pn "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_dn0.so cronsun_amd/libcronsun_gpu_dn4k.so" --workload pernode --time-order --steps 10 || exit 1
bash tools/ab_libs.sh r4m17/c3 "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_dn0.so cronsun_amd/libcronsun_gpu_dn4k.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
