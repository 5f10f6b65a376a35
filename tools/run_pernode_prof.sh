#!/bin/bash
# Per-node benches (time order, pipelined config 3) with kernel traces: tools/run_pernode_prof.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r3_pnprof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py -k "time_ordered or async or bands" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_order -- python3 bench.py --workload pernode --time-order --steps 5 --warmup 2 --cpu-sample 0 > $O/pernode_order.json 2> $O/prof_order.err || { tail -20 $O/prof_order.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/pernode_order.json')); print('pernode --time-order', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'order %.3f' % d['kernel_ms']['time_order'], d['verified'])"
find $O/prof_order -name '*kernel_stats.csv' -exec head -4 {} \; | cut -c1-160
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -- python3 bench.py --workload config3 --steps 2 --warmup 1 --cpu-sample 0 --verify-sample 0 > $O/config3.json 2> $O/prof_c3.err || { tail -20 $O/prof_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/config3.json')); print('config3', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'])"
find $O/prof_c3 -name '*kernel_stats.csv' -exec head -12 {} \; | cut -c1-160
