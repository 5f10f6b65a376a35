#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, kernel-trace profile, PMC traffic.
#   tools/gpu_check.sh <tag> [tests] [bench] [prof] [pmc] [sq]   (default: all but sq)
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-run}
shift
STEPS=" ${*:-tests bench prof pmc} "
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { [[ "$STEPS" == *" $1 "* ]]; }
fail() { echo "FAILED: $1"; tail -40 "$2"; exit 1; }

if has tests; then
  echo "== pytest -m gpu"
  CG_TEST_RECORD_DIR=$OUT timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || fail pytest "$OUT/pytest_gpu.log"
  tail -2 "$OUT/pytest_gpu.log"
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || fail smoke "$OUT/smoke.log"
  tail -1 "$OUT/smoke.log"
fi
if has bench; then
  echo "== bench"
  timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || fail bench "$OUT/bench.err"
  cat "$OUT/bench.json"
fi
if has prof; then
  echo "== rocprofv3 kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_kt" -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --verify-sample 0 > "$OUT/bench_prof.json" 2> "$OUT/prof_kt.err" \
    || fail rocprof "$OUT/prof_kt.err"
  find "$OUT/prof_kt" -name '*kernel_stats.csv' -exec cat {} \;
fi
if has pmc; then
  echo "== rocprofv3 PMC: FETCH_SIZE and WRITE_SIZE, one pass each"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/prof_fetch" -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --verify-sample 0 > /dev/null 2> "$OUT/prof_fetch.err" \
    || fail fetch "$OUT/prof_fetch.err"
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/prof_write" -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --verify-sample 0 > /dev/null 2> "$OUT/prof_write.err" \
    || fail write "$OUT/prof_write.err"
  python3 tools/pmc_traffic.py --kt "$OUT/prof_kt" --fetch "$OUT/prof_fetch" --write "$OUT/prof_write" \
    --bench "$OUT/bench_prof.json" --out "$OUT/pmc_traffic.json"
fi
if has sq; then
  echo "== rocprofv3 PMC: SQ instruction mix"
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SALU \
    SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d "$OUT/prof_sq" -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --verify-sample 0 > /dev/null 2> "$OUT/prof_sq.err" \
    || fail sq "$OUT/prof_sq.err"
  python3 tools/pmc_traffic.py --sq "$OUT/prof_sq" --out "$OUT/sq.json"
fi
echo "== done"
