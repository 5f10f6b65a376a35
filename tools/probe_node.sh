#!/bin/bash
# Diagnostic matrix for k_node_write on the pernode workload (no parity checks):
#   CG_NODE_VARIANT=1 no gather (synthetic values), 2 no stores, 3 neither
set -o pipefail
# the probe/variant switches exist only in the diagnostic build (make -C cronsun_amd/csrc diag)
export CRONSUN_GPU_LIB=$PWD/cronsun_amd/libcronsun_gpu_diag.so
OUT=gpurun_out/${1:-probe_node}
mkdir -p "$OUT"
for v in ${VARIANTS:-0 1 2 3}; do
  CG_NODE_VARIANT=$v timeout -k 10 300 python bench.py --diagnostic --workload pernode --steps 5 --warmup 2 --cpu-sample 0 \
    > "$OUT/v$v.json" 2> "$OUT/v$v.err" || { tail -20 "$OUT/v$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/v$v.json')); print('variant $v node_write=%.3f ms step=%.3f ms' % (d['kernel_ms']['node_write'], d['ms_per_step']))"
done
