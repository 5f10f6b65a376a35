#!/bin/bash
# Per-node GPU tests (time order, placement) + pernode benches with and without
# --time-order + a kernel trace of the time-ordered run.  tools/run_time_order.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r3_to}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pernode.py "tests/test_gpu_configs.py::test_config3_sharded_ranges_place_to_unsharded" tests/test_gpu_expand.py -k "not config2_scale and not multi_year and not random_specs and not starts_near" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u bench.py --workload pernode --time-order --steps 5 --warmup 2 > $O/pernode_order.json 2> $O/pernode_order.err || { tail -20 $O/pernode_order.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/pernode_order.json')); print('pernode --time-order', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], d['kernel_ms'], d['verified'])"
timeout -k 10 400 python -u bench.py --workload pernode --steps 5 --warmup 2 > $O/pernode.json 2> $O/pernode.err || { tail -20 $O/pernode.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/pernode.json')); print('pernode', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], d['kernel_ms'], d['verified'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 bench.py --workload pernode --time-order --steps 5 --warmup 2 --cpu-sample 0 --verify-sample 0 > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-150
timeout -k 10 600 python -u bench.py --workload config3 --steps 3 --warmup 1 > $O/config3.json 2> $O/config3.err || { tail -20 $O/config3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/config3.json')); print('config3', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], {k:round(v,3) for k,v in d['kernel_ms'].items() if not isinstance(v,str)}, d['verified'])"
