#!/bin/bash
# SQ instruction-mix counters of the per-node pipeline (one PMC pass each).
set -o pipefail
OUT=gpurun_out/${1:-sq_pn}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --workload pernode --steps 2 --warmup 1 --cpu-sample 0 --verify-sample 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d "$OUT/sq1" -- python3 $B > /dev/null 2> "$OUT/sq1.err" || { tail -5 "$OUT/sq1.err"; exit 1; }
python3 tools/pmc_traffic.py --sq "$OUT/sq1" --out "$OUT/sq1.json" > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM \
  --output-format csv -d "$OUT/sq2" -- python3 $B > /dev/null 2> "$OUT/sq2.err" || { tail -5 "$OUT/sq2.err"; exit 1; }
python3 tools/pmc_traffic.py --sq "$OUT/sq2" --out "$OUT/sq2.json" > /dev/null
python3 -c "
import json
for f in ('sq1','sq2'):
    d=json.load(open('$OUT/'+f+'.json'))['kernels']
    for k in ('k_node_write','k_write_cf','k_seg_records'):
        if k in d: print(f, k, {a: round(b) for a,b in d[k].items()})
"
