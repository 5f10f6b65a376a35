#!/bin/bash
# N > 1 rehearsal of bench.py's multi-rank path on one GPU: several ranks on
# cuda:0 with gloo collectives (RCCL needs one GPU per rank; it runs on the
# driver's multi-GPU node).  tools/rehearse.sh <tag> <ranks> <workload args...>
set -o pipefail
O=gpurun_out/$1
N=$2
shift 2
mkdir -p $O
export CG_DIST_BACKEND=gloo
timeout -k 10 ${REHEARSE_LIMIT:-600} python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus $N "$@" --cpu-sample 0 > $O/line.json 2> $O/line.err || { tail -30 $O/line.err; exit 1; }
python3 tools/line.py $O/line.json
