#!/bin/bash
# the dense nodes' merge with 16-wave blocks (16384-event chunks: heavy slabs merged inline, one block per CU;
# d16) vs 8-wave (production): the >2^20-rule test on production (14 index bits), parity on d16, A/B
set -o pipefail
O=gpurun_out/r4m35
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py -k "over_2_20" > $O/pytest_prod_2_20.log 2>&1 || { tail -30 $O/pytest_prod_2_20.log; exit 1; }
tail -1 $O/pytest_prod_2_20.log
CRONSUN_GPU_LIB=cronsun_amd/libcronsun_gpu_d16.so timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py tests/test_gpu_config3_day.py -k "time or order or config3" > $O/pytest_d16.log 2>&1 || { tail -30 $O/pytest_d16.log; exit 1; }
tail -1 $O/pytest_d16.log
bash tools/ab_libs.sh r4m35/c3o "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_d16.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
bash tools/ab_libs.sh r4m35/pto "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_d16.so" --workload pernode --time-order --steps 10 || exit 1
