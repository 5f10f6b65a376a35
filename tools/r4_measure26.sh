#!/bin/bash
# ot_rank's 256-digit scan by 256 threads, one digit each (sa1: no merge spills at 128 VGPRs; sa1w5: 5 waves
# per SIMD, 96 VGPRs): parity on sa1 and sa1w5, then A/B against production (lane-0 wave scans 4 digits x NW)
set -o pipefail
O=gpurun_out/r4m26
mkdir -p $O
for L in sa1 sa1w5; do
  CRONSUN_GPU_LIB=cronsun_amd/libcronsun_gpu_$L.so timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py tests/test_gpu_config3_day.py -k "time or order or config3" > $O/pytest_$L.log 2>&1 || { tail -30 $O/pytest_$L.log; exit 1; }
  tail -1 $O/pytest_$L.log
done
bash tools/ab_libs.sh r4m26/pto "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_sa1.so cronsun_amd/libcronsun_gpu_sa1w5.so" --workload pernode --time-order --steps 10 || exit 1
bash tools/ab_libs.sh r4m26/c3o "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_sa1.so cronsun_amd/libcronsun_gpu_sa1w5.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
