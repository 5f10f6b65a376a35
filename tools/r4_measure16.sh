#!/bin/bash
# merge shape A/B: raw buffer loads (production) vs flat loads (buf0), 8-wave 8192-event merge chunks (m8), runs capped at 4 slabs (r4, m8r4)
set -o pipefail
O=gpurun_out/r4m16
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py tests/test_gpu_config3_day.py -k "time or order or config3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/ab_libs.sh r4m16/pn "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_buf0.so cronsun_amd/libcronsun_gpu_m8.so cronsun_amd/libcronsun_gpu_m8r4.so cronsun_amd/libcronsun_gpu_r4.so" --workload pernode --time-order --steps 10 || exit 1
bash tools/ab_libs.sh r4m16/c3 "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_buf0.so cronsun_amd/libcronsun_gpu_m8.so cronsun_amd/libcronsun_gpu_m8r4.so cronsun_amd/libcronsun_gpu_r4.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1

