#!/bin/bash
# Kernel trace + HBM traffic of one bench line: rocprofv3 --kernel-trace
# --stats, then one FETCH_SIZE and one WRITE_SIZE pass (one counter per run),
# summarised per kernel by pmc_traffic.py (gfx950 read-side x2 correction).
#   tools/pmc.sh <tag> <bench args...>
#     -> gpurun_out/<tag>/{prof_kt,prof_fetch,prof_write,bench_prof.json,pmc_traffic.json}
#   PMC_SQ="SQ_A SQ_B ..." adds a pass of those SQ counters (<= 8) -> pmc_sq.json
#   PMC_LIMIT=<s> each pass's time limit (default 400)
set -o pipefail
O=gpurun_out/$1
shift
mkdir -p "$O"
export TMPDIR=/tmp
B="bench.py $* --cpu-sample 0 --verify-sample 0"
L=${PMC_LIMIT:-400}
timeout -k 10 $L rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -- python3 $B > $O/bench_prof.json 2> $O/kt.err || { tail -5 $O/kt.err; exit 1; }
timeout -s KILL $L rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -- python3 $B > /dev/null 2> $O/fetch.err || { tail -5 $O/fetch.err; exit 1; }
timeout -s KILL $L rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -- python3 $B > /dev/null 2> $O/write.err || { tail -5 $O/write.err; exit 1; }
python3 tools/pmc_traffic.py --kt $O/prof_kt --fetch $O/prof_fetch --write $O/prof_write --bench $O/bench_prof.json --out $O/pmc_traffic.json > /dev/null || exit 1
if [ -n "$PMC_SQ" ]; then
  timeout -s KILL $L rocprofv3 --pmc $PMC_SQ --output-format csv -d $O/prof_sq -- python3 $B > /dev/null 2> $O/sq.err || { tail -5 $O/sq.err; exit 1; }
  python3 tools/pmc_traffic.py --sq $O/prof_sq --out $O/pmc_sq.json > /dev/null || exit 1
fi
python3 - $O <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + '/pmc_traffic.json'))
ks = sorted(d['kernels'].items(), key=lambda kv: -kv[1].get('total_ns', 0))
for k, v in ks[:14]:
    print('%-40s calls %5s avg ms %8.3f  GB/launch %7.3f' % (k[:40], v.get('calls'), v.get('avg_ns', 0) / 1e6,
                                                             v.get('hbm_bytes_per_launch', 0) / 1e9))
PY
