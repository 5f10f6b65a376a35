#!/bin/bash
# merge / k_ot_big ranks with RUNS (one LDS add per run of equal digits in neighbouring lanes): parity on mr1, A/B
set -o pipefail
O=gpurun_out/r4m18
mkdir -p $O
CRONSUN_GPU_LIB=cronsun_amd/libcronsun_gpu_mr1.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py tests/test_gpu_config3_day.py -k "time or order or config3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/ab_libs.sh r4m18/pn "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_mr1.so" --workload pernode --time-order --steps 10 || exit 1
bash tools/ab_libs.sh r4m18/c3 "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_mr1.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
