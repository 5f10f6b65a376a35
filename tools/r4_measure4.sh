#!/bin/bash
# Writer layout A/B on config 2, then the config3 --time-order kernel trace + PMC traffic
set -o pipefail
bash tools/ab_libs.sh r4m4/ab "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_s10.so cronsun_amd/libcronsun_gpu_pl.so cronsun_amd/libcronsun_gpu_w2.so cronsun_amd/libcronsun_gpu_w8.so" --steps 30 --warmup 5 || exit 1
bash tools/pmc_config3_order.sh r4m4/pmc_c3o || exit 1
