"""bench.py at N = 2 on one GPU, launched by bench.py itself (`--gpus 2`, no
external launcher): two ranks over gloo, each expanding its job-ID range of
the pernode workload in (time, rule) order, the whole per-node CSR gathered on
rank 0 every timed step (shard.gather_node_csr, chunked) and, after the timed
region, the verified time-ordered gather of `verify.gather` (24 nodes against
the oracle).  The same path an 8-GPU node runs with RCCL (there through the
library's communicator, tests/test_gpu_comm.py::test_comm_world2_one_gpu)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_gather():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CG_DIST_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "pernode",
                        "--time-order", "--gather-node-csr", "--steps", "1", "--warmup", "1", "--verify-sample", "500"],
                       capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["verified"] is True
    assert d["config"]["gathered_per_node_csr_on_rank0_events"] > 0
    g = d["verify"]["gather"]
    assert g["verified"] and g["mismatched_nodes"] == 0 and g["offsets_consistent"]
    assert g["chunks"] > 100 and g["split_node_chunks"] > 0
