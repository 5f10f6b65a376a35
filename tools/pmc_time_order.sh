#!/bin/bash
# HBM traffic of the time-ordered per-node path (pernode --time-order): kernel trace, then FETCH_SIZE and
# WRITE_SIZE passes, summarised per kernel.  tools/pmc_time_order.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r3_pmc_to}
mkdir -p $O
export TMPDIR=/tmp
B="bench.py --workload pernode --time-order --steps 3 --warmup 4 --cpu-sample 0 --verify-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -- python3 $B > $O/bench_prof.json 2> $O/kt.err || { tail -5 $O/kt.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -- python3 $B > /dev/null 2> $O/fetch.err || { tail -5 $O/fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -- python3 $B > /dev/null 2> $O/write.err || { tail -5 $O/write.err; exit 1; }
python3 tools/pmc_traffic.py --kt $O/prof_kt --fetch $O/prof_fetch --write $O/prof_write --bench $O/bench_prof.json --out $O/pmc_traffic.json
python3 - $O <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + '/pmc_traffic.json'))
for k in ('k_node_write', 'k_ot_tile', 'k_ot_slabs', 'k_ot_merge', 'k_ot_big', 'k_seg_records'):
    if k in d['kernels']:
        v = d['kernels'][k]
        print(k, 'avg ms %.3f' % (v['avg_ns'] / 1e6), 'GB/launch %.3f' % (v['hbm_bytes_per_launch'] / 1e9))
PY
