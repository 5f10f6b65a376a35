#!/bin/bash
# the sparse merge's items per thread (with the all-thread scan): 16 at 4 waves/SIMD (production), 8 at 6 (it8:
# 2048-event chunks, 80 VGPRs), 12 at 5 (it12: 3072-event chunks, 96 VGPRs), no spills in any: parity, A/B
set -o pipefail
O=gpurun_out/r4m32
mkdir -p $O
for L in it8 it12; do
  CRONSUN_GPU_LIB=cronsun_amd/libcronsun_gpu_$L.so timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py -k "time or order" > $O/pytest_$L.log 2>&1 || { tail -30 $O/pytest_$L.log; exit 1; }
  tail -1 $O/pytest_$L.log
done
bash tools/ab_libs.sh r4m32/pto "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_it8.so cronsun_amd/libcronsun_gpu_it12.so" --workload pernode --time-order --steps 10 || exit 1
bash tools/ab_libs.sh r4m32/c3o "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_it8.so cronsun_amd/libcronsun_gpu_it12.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
