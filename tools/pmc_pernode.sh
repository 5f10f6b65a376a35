#!/bin/bash
# PMC traffic of the per-node pipeline (bench --workload pernode): kernel
# trace, FETCH_SIZE and WRITE_SIZE passes, summarised per kernel.
#   tools/pmc_pernode.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-pn}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --workload pernode --steps 3 --warmup 1 --cpu-sample 0 --verify-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_kt" -- \
  python3 $B > "$OUT/bench_prof.json" 2> "$OUT/prof_kt.err" || { tail -20 "$OUT/prof_kt.err"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/prof_fetch" -- \
  python3 $B > /dev/null 2> "$OUT/prof_fetch.err" || { tail -20 "$OUT/prof_fetch.err"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/prof_write" -- \
  python3 $B > /dev/null 2> "$OUT/prof_write.err" || { tail -20 "$OUT/prof_write.err"; exit 1; }
python3 tools/pmc_traffic.py --kt "$OUT/prof_kt" --fetch "$OUT/prof_fetch" --write "$OUT/prof_write" \
  --bench "$OUT/bench_prof.json" --out "$OUT/pmc_traffic.json"
find "$OUT/prof_kt" -name '*kernel_stats.csv' -exec cat {} \;
