#!/bin/bash
# Interleaved A/B of two in-tree builds (A: cronsun_amd/libcronsun_gpu_A.so, B: the default library) on
# one bench line.  tools/ab_lib.sh <tag> <bench args...>
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
for v in A B A B; do
  L=cronsun_amd/libcronsun_gpu.so; [ $v = A ] && L=cronsun_amd/libcronsun_gpu_A.so
  CRONSUN_GPU_LIB=$L timeout -k 10 300 python -u bench.py "$@" --cpu-sample 0 --verify-sample 250 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.json')); k=d['kernel_ms']; print('$v', 'step %.3f' % d['ms_per_step'], {a: round(b, 3) for a, b in k.items() if isinstance(b, float) and b > 0.05}, d['verified'])" | tee -a $O/summary.txt
done
