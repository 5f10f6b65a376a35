#!/bin/bash
# Time-ordered per-node writer: its GPU tests, then pernode benches (direct time order, pipelined,
# and the separate pass for comparison) with a kernel trace.  tools/run_timed.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r3_tw}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pernode.py -k "time_ordered or async" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 bench.py --workload pernode --time-order --steps 5 --warmup 2 --cpu-sample 0 > $O/pernode_timed.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/pernode_timed.json')); print('pernode --time-order', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], d['kernel_ms'].get('node_write'), d['verified'], d.get('steps_mode'))"
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/prof/**/*kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r['Name'][:50].ljust(50), r['Calls'], '%.3f ms' % (float(r['AverageNs']) / 1e6))
PY
