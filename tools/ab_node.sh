#!/bin/bash
# A/B of per-node writer builds (diagnostic libraries): node_write time per
# build and blocks-per-CU setting.  tools/ab_node.sh <tag> "<lib suffixes>" "<blocks per CU>"
set -o pipefail
OUT=gpurun_out/${1:-ab_node}
mkdir -p "$OUT"
for v in ${2:-diag}; do
  for b in ${3:-8}; do
    CRONSUN_GPU_LIB=$PWD/cronsun_amd/libcronsun_gpu_$v.so CG_NODE_BLOCKS_PER_CU=$b timeout -k 10 300 \
      python bench.py --diagnostic --workload pernode --steps 5 --warmup 2 --cpu-sample 0 --verify-sample 0 \
      > "$OUT/${v}_b$b.json" 2> "$OUT/${v}_b$b.err" || { tail -20 "$OUT/${v}_b$b.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v}_b$b.json')); print('$v blocks/CU $b node_write=%.3f ms step=%.3f ms' % (d['kernel_ms']['node_write'], d['ms_per_step']))"
  done
done
