#!/bin/bash
# Per-node GPU tests, then an interleaved pernode A/B (cronsun_amd/libcronsun_gpu_A.so vs the default
# library) and config 3 with each.  tools/run_pn_ab.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r3_pnab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pernode.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_libs.sh ${1:-r3_pnab} "cronsun_amd/libcronsun_gpu_A.so cronsun_amd/libcronsun_gpu.so" --workload pernode --steps 20 --warmup 4 || exit 1
for L in cronsun_amd/libcronsun_gpu_A.so cronsun_amd/libcronsun_gpu.so; do
  CRONSUN_GPU_LIB=$L timeout -k 10 300 python -u bench.py --workload config3 --steps 2 --warmup 2 --cpu-sample 0 > $O/c3_$(basename $L .so).json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$(basename $L .so).json')); print('config3 $L', 'step %.3f' % d['ms_per_step'], 'node_write %.3f' % d['kernel_ms']['node_write'], d['verified'])"
done
