#!/bin/bash
# A/B of k_write_cf's round-robin share of position slices (CG_WRITE_STATIC, diagnostic library):
# config 2 and config 4.  tools/ab_static.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r3_abs}
mkdir -p $O
for wl in config2 config4; do
  for pct in 0 80 90 97 0 80 90 97; do
    steps=20; [ $wl = config4 ] && steps=4
    CRONSUN_GPU_LIB=cronsun_amd/libcronsun_gpu_diag.so CG_WRITE_STATIC=$pct timeout -k 10 300 python -u bench.py --workload $wl --diagnostic --steps $steps --warmup 2 --cpu-sample 0 --verify-sample 300 > $O/$wl.$pct.json 2> $O/$wl.$pct.err || { tail -5 $O/$wl.$pct.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$wl.$pct.json')); print('$wl', 'static $pct%', 'step %.4f' % d['ms_per_step'], 'write_cf %.4f' % d['kernel_ms']['write_cf'], 'frac %.3f' % d['roofline']['frac'], d['verified'])" | tee -a $O/summary.txt
  done
done
