#!/bin/bash
# Round-4 final (g): rocprof kernel stats + PMC traffic of the headline on the final tree -> gpurun_out/r4fg
set -o pipefail
O=gpurun_out/r4fg
mkdir -p $O
export TMPDIR=/tmp
B="bench.py --steps 20 --warmup 5 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -- python3 $B > $O/bench_prof.json 2> $O/kt.err || { tail -5 $O/kt.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -- python3 $B > /dev/null 2> $O/fetch.err || { tail -5 $O/fetch.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -- python3 $B > /dev/null 2> $O/write.err || { tail -5 $O/write.err; exit 1; }
python3 tools/pmc_traffic.py --kt $O/prof_kt --fetch $O/prof_fetch --write $O/prof_write --bench $O/bench_prof.json --out $O/pmc_traffic.json
