#!/bin/bash
# overlapped time-ordered windows (window k's merges on their own stream beside window k+1's writer and tile
# sort): the per-node / config-3 / comm / fixture GPU tests, then A/B against ov0 (merges on the writer's stream)
set -o pipefail
O=gpurun_out/r4m28
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py tests/test_gpu_config3_day.py tests/test_gpu_comm.py tests/test_rule_nodes_fixtures.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/ab_libs.sh r4m28/pto "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_ov0.so" --workload pernode --time-order --steps 10 || exit 1
bash tools/ab_libs.sh r4m28/c3o "cronsun_amd/libcronsun_gpu.so cronsun_amd/libcronsun_gpu_ov0.so" --workload config3 --time-order --steps 1 --warmup 1 || exit 1
