#!/bin/bash
# k_seg_records pairs per lane (VGPRs -> waves beside the pipelined node writer): pernode / config3 A/B
set -o pipefail
bash tools/ab_libs.sh r4m14/pn "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_sp4.so cronsun_amd/libcronsun_gpu_sp6.so" --workload pernode --steps 20 || exit 1
bash tools/ab_libs.sh r4m14/c3 "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_sp4.so cronsun_amd/libcronsun_gpu_sp6.so" --workload config3 --steps 2 --warmup 1 || exit 1
