#!/bin/bash
# N = 2 rehearsal of bench.py's multi-rank path on one GPU: gloo collectives, both ranks on cuda:0
# (RCCL runs only on the driver's multi-GPU node).  tools/n2_rehearsal.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r3_n2}
mkdir -p $O
export CG_DIST_BACKEND=gloo
for wl in config2 pernode config4; do
  st=6; [ $wl = config4 ] && st=2
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --workload $wl --steps $st --warmup 3 --cpu-sample 0 --verify-sample 300 > $O/$wl.json 2> $O/$wl.err || { tail -30 $O/$wl.err; exit 1; }
  python3 -c "import json; d=json.loads([x for x in open('$O/$wl.json') if x.startswith('{')][-1]); print('$wl n=2 gloo', '%.4g' % d['value'], d['unit'], 'ms/step %.3f' % d['ms_per_step'], 'verified', d.get('verified'), (d.get('verify') or {}).get('verified_all_ranks'))"
done
