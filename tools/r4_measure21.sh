#!/bin/bash
# kernel traces + HBM traffic of both time-order lines after the packed words
set -o pipefail
bash tools/pmc_config3_order.sh r4m21/c3o || exit 1
bash tools/pmc_time_order.sh r4m21/pto || exit 1
