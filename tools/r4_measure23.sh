#!/bin/bash
# the time-order writer's packed runs stepped in 32 bits (production) vs the generic 64-bit path (pr0): parity, A/B
set -o pipefail
O=gpurun_out/r4m23
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py tests/test_gpu_config3_day.py -k "time or order or config3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/ab_libs.sh r4m23/pto "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_pr0.so" --workload pernode --time-order --steps 10 || exit 1
bash tools/ab_libs.sh r4m23/c3o "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_pr0.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
