#!/bin/bash
# packed time-order words (writer -> tile -> merge as offset << 20 | rule, 4 B instead of 2 + 4): parity,
# then A/B against pin0 (16-bit offsets + rules, same tree) and head (the previous commit) on the time-order
# and rule-order per-node lines (the writer's store lambda changed its register use: 42 -> 34 VGPRs)
set -o pipefail
O=gpurun_out/r4m20
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py tests/test_gpu_config3_day.py tests/test_gpu_comm.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/ab_libs.sh r4m20/pto "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_pin0.so cronsun_amd/libcronsun_gpu_head.so" --workload pernode --time-order --steps 10 || exit 1
bash tools/ab_libs.sh r4m20/pn "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_head.so" --workload pernode --steps 20 || exit 1
bash tools/ab_libs.sh r4m20/c3o "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_pin0.so cronsun_amd/libcronsun_gpu_head.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
