#!/bin/bash
# config3 --time-order kernel trace + HBM traffic; SQ counters of the time-order kernels (pernode --time-order)
set -o pipefail
bash tools/pmc_config3_order.sh r4m13/c3o || exit 1
bash tools/sq_time_order.sh r4m13/sq || exit 1
