#!/bin/bash
# k_write_cf store batch at the 80-VGPR cap: 8 (production, 148 B spill), 6 (88 B), 4 (52 B); config 2 headline
set -o pipefail
bash tools/ab_libs.sh r4m24/ab "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_b6.so cronsun_amd/libcronsun_gpu_b4.so" --steps 30 --warmup 5 || exit 1
