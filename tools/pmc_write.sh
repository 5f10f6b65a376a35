#!/bin/bash
# Diagnostic PMC passes on k_write_cf vs the plain-fill probe (one counter group per run).
set -o pipefail
# the probe/variant switches exist only in the diagnostic build (make -C cronsun_amd/csrc diag)
export CRONSUN_GPU_LIB=$PWD/cronsun_amd/libcronsun_gpu_diag.so
export TMPDIR=/tmp
O=gpurun_out/pmcw
mkdir -p $O
pass() {  # name counters... (env via PMC_ENV)
  local name=$1; shift
  env $PMC_ENV timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -- \
    python3 bench.py --diagnostic --steps 3 --warmup 1 --cpu-sample 0 > /dev/null 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  python3 tools/pmc_traffic.py --sq $O/$name --out $O/$name.json > /dev/null
  python3 -c "import json; d=json.load(open('$O/$name.json'))['kernels']; k=d.get('k_write_cf') or d.get('k_fill_probe'); print('$name', json.dumps(k))"
}
for mode in base fill16; do
  case $mode in
    base) PMC_ENV="X=0";;
    fill16) PMC_ENV="CG_WRITE_PROBE=2";;
  esac
  pass ${mode}_sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU
done
