#!/bin/bash
# The whole -m gpu suite (one process) + smoke + the headline bench; logs under gpurun_out/<tag>
set -o pipefail
O=gpurun_out/${1:-r4_suite}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('config2 %.4g' % d['value'], 'ms %.3f' % d['ms_per_step'], 'write_cf %.3f' % d['kernel_ms']['write_cf'], 'frac %.3f' % r['frac'], 'ceil %.3f' % r['store_ceiling']['frac_of_ceiling'], d['verified'])"
