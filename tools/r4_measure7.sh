#!/bin/bash
# Writer launch-bound A/B: production (2-wave x 6, 3 waves/SIMD bound), w2s (the same with a 6 waves/SIMD bound: spills), w4 (4-wave x 3)
set -o pipefail
bash tools/ab_libs.sh r4m7/ab "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_w2s.so cronsun_amd/libcronsun_gpu_w4.so" --steps 30 --warmup 5 || exit 1
