#!/bin/bash
# k_ot_mid's 16-wave form for slabs of 8193..16384 events (instead of k_ot_big): parity, A/B against m2off
set -o pipefail
O=gpurun_out/r4m19
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py tests/test_gpu_config3_day.py -k "time or order or config3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/ab_libs.sh r4m19/c3 "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_m2off.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
bash tools/ab_libs.sh r4m19/pn "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_m2off.so" --workload pernode --time-order --steps 10 || exit 1
