#!/bin/bash
# Phase clocks of the time-ordered per-node kernels (diagnostic library, synchronous windows), then the
# production pipelined bench with a kernel trace.  tools/prof_timed.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r3_pt}
mkdir -p $O
export TMPDIR=/tmp
CRONSUN_GPU_LIB=cronsun_amd/libcronsun_gpu_diag.so timeout -k 10 300 python -u bench.py --workload pernode --time-order --sync --diagnostic --steps 2 --warmup 1 --cpu-sample 0 --verify-sample 0 > $O/diag.json 2> $O/diag.err || { tail -20 $O/diag.err; exit 1; }
grep -E "k_seg_tiles|k_ot_merge" $O/diag.err | tail -2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 bench.py --workload pernode --time-order --steps 5 --warmup 2 --cpu-sample 0 > $O/pernode_timed.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/pernode_timed.json')); print('pernode --time-order', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], d['kernel_ms'].get('node_write'), d['verified'])"
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/prof/**/*kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:6]:
    print(r['Name'][:50].ljust(50), r['Calls'], '%.3f ms' % (float(r['AverageNs']) / 1e6))
PY
