#!/bin/bash
# Writer layout A/B round 2 (config 2), then config3 --time-order kernel trace + PMC
set -o pipefail
bash tools/ab_libs.sh r4m6/ab "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_w2.so cronsun_amd/libcronsun_gpu_w2b5.so cronsun_amd/libcronsun_gpu_w1b12.so cronsun_amd/libcronsun_gpu_b16.so cronsun_amd/libcronsun_gpu_b4.so cronsun_amd/libcronsun_gpu_tg64.so cronsun_amd/libcronsun_gpu_tg16.so" --steps 30 --warmup 5 || exit 1
bash tools/pmc_config3_order.sh r4m6/pmc_c3o || exit 1
