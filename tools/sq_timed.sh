#!/bin/bash
# SQ counters of the time-ordered per-node kernels (k_ot_tile, k_ot_merge), two PMC passes.  tools/sq_timed.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-sq_tw}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --workload pernode --time-order --steps 2 --warmup 1 --cpu-sample 0 --verify-sample 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d "$OUT/sq1" -- python3 $B > /dev/null 2> "$OUT/sq1.err" || { tail -5 "$OUT/sq1.err"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  --output-format csv -d "$OUT/sq2" -- python3 $B > /dev/null 2> "$OUT/sq2.err" || { tail -5 "$OUT/sq2.err"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + '/sq*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        for kn in ('k_ot_tile', 'k_ot_merge', 'k_seg_records', 'k_node_write'):
            if kn in r['Kernel_Name']:
                tot[kn, r['Counter_Name']] += float(r['Counter_Value'])
                n[kn, r['Counter_Name']] += 1
for k in sorted(tot): print(k[0], k[1], '%.4g' % (tot[k] / max(1, n[k])))
PY
