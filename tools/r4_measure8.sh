#!/bin/bash
# k_write_cf register cap (min waves per SIMD bound) A/B, 2-wave blocks x 6 per CU
set -o pipefail
bash tools/ab_libs.sh r4m8/ab "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_wpe4.so cronsun_amd/libcronsun_gpu_wpe5.so cronsun_amd/libcronsun_gpu_w2s.so cronsun_amd/libcronsun_gpu_wpe8.so" --steps 30 --warmup 5 || exit 1
