#!/bin/bash
# L2 hit/miss of the per-node pipeline's kernels (one PMC pass):
#   tools/pmc_l2_pernode.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-l2_pn}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --workload pernode --steps 2 --warmup 1 --cpu-sample 0 --verify-sample 0"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/l2" -- python3 $B \
  > /dev/null 2> "$OUT/l2.err" || { tail -5 "$OUT/l2.err"; exit 1; }
python3 - "$OUT" <<'PY'
import sys, csv, glob, collections, re
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for p in glob.glob(out + "/l2/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        m = re.search(r"\b(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:30]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r.get("Dispatch_Id", ""))
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("TCC_HIT_sum", 0)):
    h, m = v.get("TCC_HIT_sum", 0) / len(n[k]), v.get("TCC_MISS_sum", 0) / len(n[k])
    print(f"{k:24s} hit {h:.3e} miss {m:.3e} hit-rate {h / max(h + m, 1):.3f}")
PY
