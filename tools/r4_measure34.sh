#!/bin/bash
# dense-merge threshold 2048 (dn2k) vs 4096 (production): config3 --time-order, and pernode --time-order again
set -o pipefail
bash tools/ab_libs.sh r4m34/c3o "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_dn2k.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
bash tools/ab_libs.sh r4m34/pto "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_dn2k.so" --workload pernode --time-order --steps 10 || exit 1
