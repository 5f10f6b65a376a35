#!/bin/bash
# The whole -m gpu suite (one process) + smoke() + the headline bench line.
#   tools/suite.sh <tag> [pytest -k expression]   -> gpurun_out/<tag>/{pytest.log,smoke.log,bench.json}
set -o pipefail
O=gpurun_out/${1:-suite}
mkdir -p $O
K=${2:+-k "$2"}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread $K > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 tools/line.py $O/bench.json
