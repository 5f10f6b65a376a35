#!/bin/bash
# dense-merge threshold with the all-thread scan (no merge spills): 4096 (production) vs 3584 vs 3072 events per slab
set -o pipefail
bash tools/ab_libs.sh r4m27/pto "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_dn35.so cronsun_amd/libcronsun_gpu_dn3k.so" --workload pernode --time-order --steps 10 || exit 1
bash tools/ab_libs.sh r4m27/c3o "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_dn35.so cronsun_amd/libcronsun_gpu_dn3k.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
