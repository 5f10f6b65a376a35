#!/bin/bash
# the dense merge's persistent grid: 2 blocks per CU (production) vs 1 and 3
set -o pipefail
bash tools/ab_libs.sh r4m29/c3o "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_db1.so cronsun_amd/libcronsun_gpu_db3.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
