#!/bin/bash
# SQ counters of the time-order pass (pernode --time-order): tools/pmc_timed.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r3_pmc_timed}
mkdir -p $O
export TMPDIR=/tmp
B="bench.py --workload pernode --time-order --steps 2 --warmup 1 --cpu-sample 0 --verify-sample 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/p1 -- python3 $B > /dev/null 2> $O/p1.err || { tail -5 $O/p1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/p2 -- python3 $B > /dev/null 2> $O/p2.err || { tail -5 $O/p2.err; exit 1; }
for p in p1 p2; do
  f=$(find $O/$p -name '*counter_collection.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    kn = next((x for x in ('k_ot_tile', 'k_ot_merge', 'k_ot_big', 'k_node_write') if x in r['Kernel_Name']), None)
    if kn is None: continue
    k = kn + ':' + r['Counter_Name']
    agg[k] += float(r['Counter_Value']); n[k] += 1
for k in sorted(agg): print(k, '%.4g' % (agg[k] / max(1, n[k]) * 1), 'per-dispatch-avg(sum over rows/dispatch rows)')
PY
done
