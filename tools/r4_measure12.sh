#!/bin/bash
# packed tile sort (k_ot_tile<.., PACK>: no LDS rule array, 6 waves per SIMD): time-order parity, then
# A/B against tp0 (the LDS rule array) and tw5 (packed, 5 waves per SIMD)
set -o pipefail
O=gpurun_out/r4m12
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py tests/test_gpu_config3_day.py -k "time or order or config3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/ab_libs.sh r4m12/pn "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_tp0.so cronsun_amd/libcronsun_gpu_tw5.so" --workload pernode --time-order --steps 10 || exit 1
bash tools/ab_libs.sh r4m12/c3 "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_tp0.so cronsun_amd/libcronsun_gpu_tw5.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
