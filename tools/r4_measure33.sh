#!/bin/bash
# dense-merge threshold again after the all-thread scan removed the 8-wave merge's spills: 4096 (production)
# vs 2048 and 1024 events per slab (pernode's nodes average ~1.6 k): pernode --time-order
set -o pipefail
bash tools/ab_libs.sh r4m33/pto "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_dn2k.so cronsun_amd/libcronsun_gpu_dn1k.so" --workload pernode --time-order --steps 10 || exit 1
