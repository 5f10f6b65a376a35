#!/bin/bash
# Diagnostic: time k_write_cf variants (CG_ABLATE) on the bench workload.
#   0 normal, 1 no global stores, 2 stores only, 3 locate only, 4 hipMemset of the same bytes
for m in 0 1 3 4; do
  CG_ABLATE=$m timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ABLATE=$m', 'write_cf_ms=%.3f' % d['kernel_ms']['write_cf'], 'count_ms=%.3f' % d['kernel_ms']['count'], 'events=%d' % d['config']['events_per_gpu_step'])" || exit 1
done
