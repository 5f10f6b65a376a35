#!/bin/bash
# k_write_cf slice size with the 2-wave x 6 layout: 2048 events (production) vs 4096 (s12); config 2 headline
set -o pipefail
bash tools/ab_libs.sh r4m31/ab "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_s12.so" --steps 30 --warmup 5 || exit 1
