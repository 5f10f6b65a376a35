#!/bin/bash
# Round-4 final (c): the other workloads' bench lines after the time-order work (CPU baselines included)
# -> gpurun_out/r4fc, then the config3 --time-order kernel trace + HBM traffic -> gpurun_out/r4fc/c3o
set -o pipefail
sed 's#O=gpurun_out/r4fb#O=gpurun_out/r4fc#' tools/r4_final_b.sh > /tmp/r4_final_c_b.sh
bash /tmp/r4_final_c_b.sh || exit 1
bash tools/pmc_config3_order.sh r4fc/c3o || exit 1
