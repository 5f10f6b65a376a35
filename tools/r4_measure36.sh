#!/bin/bash
# dense-merge threshold around 2048: 1536 / 2048 (production) / 2560 events per slab, pernode --time-order
set -o pipefail
bash tools/ab_libs.sh r4m36/pto "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_dn15.so cronsun_amd/libcronsun_gpu_dn25.so" --workload pernode --time-order --steps 10 || exit 1
