#!/bin/bash
# Store ceiling on the config-2 output: the writer vs plain fills of the same
# E*8 bytes with the same grid and slices (CG_WRITE_PROBE: 1 = 8 B/lane,
# 2 = 16 B/lane, 5 = hipMemsetAsync of the capacity).  No parity checks.
set -o pipefail
# the probe/variant switches exist only in the diagnostic build (make -C cronsun_amd/csrc diag)
export CRONSUN_GPU_LIB=$PWD/cronsun_amd/libcronsun_gpu_diag.so
OUT=gpurun_out/${1:-probe_fill}
mkdir -p "$OUT"
for round in 1 2; do
  for pr in ${PROBES:-0 1 2 5}; do
    CG_WRITE_PROBE=$pr timeout -k 10 300 python bench.py --diagnostic --steps 20 --warmup 3 --cpu-sample 0 \
      > "$OUT/p${pr}_$round.json" 2> "$OUT/p${pr}_$round.err" || { tail -20 "$OUT/p${pr}_$round.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/p${pr}_$round.json')); print('probe $pr r$round write_cf=%.4f ms' % d['kernel_ms']['write_cf'])"
  done
done
