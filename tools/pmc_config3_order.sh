#!/bin/bash
# Kernel trace + HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of config3 --time-order: 1M jobs x 10k nodes,
# config-2 mix, 24 one-hour windows in (time, rule) order.  tools/pmc_config3_order.sh <tag> [extra bench args]
set -o pipefail
O=gpurun_out/${1:-r4_pmc_c3o}
shift
mkdir -p $O
export TMPDIR=/tmp
B="bench.py --workload config3 --time-order --steps 1 --warmup 1 --cpu-sample 0 --verify-sample 0 $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -- python3 $B > $O/bench_prof.json 2> $O/kt.err || { tail -5 $O/kt.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -- python3 $B > /dev/null 2> $O/fetch.err || { tail -5 $O/fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -- python3 $B > /dev/null 2> $O/write.err || { tail -5 $O/write.err; exit 1; }
python3 tools/pmc_traffic.py --kt $O/prof_kt --fetch $O/prof_fetch --write $O/prof_write --bench $O/bench_prof.json --out $O/pmc_traffic.json
python3 - $O <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + '/pmc_traffic.json'))
for k, v in sorted(d['kernels'].items(), key=lambda kv: -kv[1].get('avg_ns', 0) * kv[1].get('calls', 0)):
    print(k, 'calls', v.get('calls'), 'avg ms %.3f' % (v.get('avg_ns', 0) / 1e6), 'GB/launch %.3f' % (v.get('hbm_bytes_per_launch', 0) / 1e9))
PY
