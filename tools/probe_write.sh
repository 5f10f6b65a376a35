#!/bin/bash
# Diagnostic matrix for k_write_cf on the bench workload (no parity checks):
#   CG_WRITE_PROBE=1/2   plain fill of the same bytes (8/16 B per lane): store ceiling
#   CG_WRITE_VARIANT=255 the loader/writer split k_write_lw (cg_diag.hip)
#   CG_WRITE_BLOCKS_PER_CU  persistent grid size
set -o pipefail
# the probe/variant switches exist only in the diagnostic build (make -C cronsun_amd/csrc diag)
export CRONSUN_GPU_LIB=$PWD/cronsun_amd/libcronsun_gpu_diag.so
mkdir -p gpurun_out/probe
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --diagnostic --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/probe/$name.json 2> gpurun_out/probe/$name.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/probe/$name.json')); print('%-14s write_cf_ms=%.4f' % ('$name', d['kernel_ms']['write_cf']))"
}
run base X=0
run b4 CRONSUN_GPU_LIB=$PWD/cronsun_amd/libcronsun_gpu_b4.so
run fill8 CG_WRITE_PROBE=1
run base2 X=0
run b4_2 CRONSUN_GPU_LIB=$PWD/cronsun_amd/libcronsun_gpu_b4.so
