#!/bin/bash
set -o pipefail
bash tools/ab_libs.sh r4m10/ab "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_w2b8.so cronsun_amd/libcronsun_gpu_w2b5.so cronsun_amd/libcronsun_gpu_wpe7.so cronsun_amd/libcronsun_gpu_w4wpe6.so" --steps 30 --warmup 5 || exit 1
