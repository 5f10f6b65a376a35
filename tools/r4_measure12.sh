#!/bin/bash
# config3 --time-order kernel trace + HBM traffic with k_ot_mid; SQ counters of the time-order kernels
set -o pipefail
bash tools/pmc_config3_order.sh r4m12/c3o || exit 1
bash tools/sq_time_order.sh r4m12/sq || exit 1
