#!/bin/bash
# Per-node pipelined benches (pernode, pernode --time-order, config3) with kernel traces: tools/run_pn_pipe.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r3_pp}
mkdir -p $O
export TMPDIR=/tmp
for args in "pernode" "pernode --time-order" "config3"; do
  tag=$(echo $args | tr -d ' -')
  st=8; [ "$args" = config3 ] && st=2
  timeout -k 10 400 python -u bench.py --workload $args --steps $st --warmup 2 > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$args', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'node_write %.3f' % d['kernel_ms']['node_write'], d['verified'], 'frac %.3f' % d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 bench.py --workload pernode --steps 8 --warmup 2 --cpu-sample 0 --verify-sample 0 > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/prof/**/*kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
last = [r for r in rows if 'k_node_write' in r['Kernel_Name']][-6:]
t0 = int(last[0]['Start_Timestamp'])
for r in rows:
    s = int(r['Start_Timestamp'])
    if s >= t0 - 2_000_000 and s <= int(last[-1]['End_Timestamp']):
        print('%9.1f %9.1f us  %s' % ((s - t0) / 1e3, (int(r['End_Timestamp']) - s) / 1e3, r['Kernel_Name'][:60]))
PY
