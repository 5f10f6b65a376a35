#!/bin/bash
# SQ instruction-mix / wait counters of the time-order kernels (pernode --time-order; one PMC pass each).
#   tools/sq_time_order.sh <tag> [extra bench args]
set -o pipefail
OUT=gpurun_out/${1:-sq_to}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --workload pernode --time-order --steps 2 --warmup 1 --cpu-sample 0 --verify-sample 0 $*"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d "$OUT/sq1" -- python3 $B > /dev/null 2> "$OUT/sq1.err" || { tail -5 "$OUT/sq1.err"; exit 1; }
python3 tools/pmc_traffic.py --sq "$OUT/sq1" --out "$OUT/sq1.json" > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM \
  --output-format csv -d "$OUT/sq2" -- python3 $B > /dev/null 2> "$OUT/sq2.err" || { tail -5 "$OUT/sq2.err"; exit 1; }
python3 tools/pmc_traffic.py --sq "$OUT/sq2" --out "$OUT/sq2.json" > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH \
  --output-format csv -d "$OUT/sq3" -- python3 $B > /dev/null 2> "$OUT/sq3.err" || { tail -5 "$OUT/sq3.err"; exit 1; }
python3 tools/pmc_traffic.py --sq "$OUT/sq3" --out "$OUT/sq3.json" > /dev/null
python3 -c "
import json
for f in ('sq1','sq2','sq3'):
    d=json.load(open('$OUT/'+f+'.json'))['kernels']
    for k in ('k_node_write','k_ot_tile','k_ot_merge','k_ot_mid','k_ot_big'):
        if k in d: print(f, k, {a: round(b) for a,b in d[k].items()})
"
