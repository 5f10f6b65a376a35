#!/bin/bash
# k_ot_mid (slabs of 4097..8192 events merged by an 8-wave chunk instead of k_ot_big):
# time-order parity, then config-3 / pernode time-order A/B against mid0 (all to k_ot_big)
set -o pipefail
O=gpurun_out/r4m11
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py tests/test_gpu_config3_day.py -k "time or order or config3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/ab_libs.sh r4m11/c3 "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_mid0.so cronsun_amd/libcronsun_gpu_mid2.so cronsun_amd/libcronsun_gpu_mid3.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
bash tools/ab_libs.sh r4m11/pn "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_mid0.so" --workload pernode --time-order --steps 10 || exit 1
