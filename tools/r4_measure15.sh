#!/bin/bash
# merge portion lookup: owner map (production) vs binary search + walk (gs2): time-order parity on gs2, then A/B
set -o pipefail
O=gpurun_out/r4m15
mkdir -p $O
CRONSUN_GPU_LIB=cronsun_amd/libcronsun_gpu_gs2.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py -k "time or order" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/ab_libs.sh r4m15/pn "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_gs2.so cronsun_amd/libcronsun_gpu_gs2w5.so" --workload pernode --time-order --steps 10 || exit 1
bash tools/ab_libs.sh r4m15/c3 "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_gs2.so cronsun_amd/libcronsun_gpu_gs2w5.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
