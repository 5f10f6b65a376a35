"""The library's RCCL exchanges behind the C-ABI (cg_comm_*, cg_comm.cpp) on
one MI355X: a world-1 communicator (one GPU per rank; RCCL refuses two ranks
on one device, so the N > 1 paths are covered by the same chunk plan in the
gloo tests, tests/test_distributed.py, and run on the driver's 8-GPU node).

World 1 runs every collective for real: the all-gather of host values, the
per-node counts all-gather behind cg_comm_node_offsets, and the gather of the
per-node CSR (root's own slice placed by the kernel into caller buffers),
plus the status every rank must agree on (capacity, no readable result), a
time-ordered result gathered in time order, and a clean exit when torch is
imported after the library loaded RCCL.  The time-ordered merge of several
ranks' slices is checked on one GPU through cg_node_csr_merge_ranks
(tests/test_gpu_pernode.py) and the C++ chunk plan against the Python one on
CPU (tests/test_distributed.py)."""
import numpy as np
import pytest

from cronsun_amd import _lib, cron, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def world1():
    from cronsun_amd.engine import Comm, Engine
    eng = Engine(0)
    comm = Comm(eng, 1, 0, Comm.unique_id())
    yield eng, comm
    comm.free()
    eng.close()


def test_allgather_i64_world1(world1):
    eng, comm = world1
    v = np.array([5, -7, 1 << 40], dtype=np.int64)
    assert np.array_equal(comm.allgather_i64(v), v[None, :])


def test_node_offsets_and_gather_world1(world1):
    import torch
    eng, comm = world1
    rin = synth.multi_rule_jobs(500, seed=77, key_choices=2)
    specs = synth.spec_mix(rin.n_rules, seed=78, mix=synth.MIX_CONFIG2)
    scheds = [cron.Parse(s) for s in specs]
    t0 = synth.T0_2026 + 5 * 86400
    node_off, time, rule = eng.expand_per_node(scheds, None, t0, t0 + 3600, rin, _lib.EXCLUDE_NONE)
    E = int(node_off[-1])
    assert E > 10000
    start, base = comm.node_offsets(rin.n_nodes)
    assert np.array_equal(base, node_off) and np.array_equal(start, node_off[:-1])
    dev = torch.device("cuda", 0)
    o = torch.empty(rin.n_nodes + 1, dtype=torch.int64, device=dev)
    t = torch.full((E,), -1, dtype=torch.int64, device=dev)
    r = torch.full((E,), -1, dtype=torch.int32, device=dev)
    for budget in (24, 1 << 30):
        t.fill_(-1)
        r.fill_(-1)
        torch.cuda.synchronize(dev)
        n = comm.gather_node_csr(0, 1000, budget, o.data_ptr(), t.data_ptr(), r.data_ptr(), E)
        assert n == E
        assert np.array_equal(o.cpu().numpy(), node_off)
        assert np.array_equal(t.cpu().numpy(), time)
        assert np.array_equal(r.cpu().numpy(), rule + 1000)  # rule_base makes rule indices global
    # too small a capacity: CG_ECAPACITY, the total still reported
    with pytest.raises(_lib.CgError) as err:
        comm.gather_node_csr(0, 0, 1 << 30, o.data_ptr(), t.data_ptr(), r.data_ptr(), E - 1)
    assert err.value.code == _lib.CG_ECAPACITY
    # a time-ordered result is gathered in time order (world 1: nothing to merge)
    eng.set_node_order(_lib.NODE_ORDER_TIME)
    try:
        node_off2, time2, rule2 = eng.expand_per_node(scheds, None, t0, t0 + 3600, rin, _lib.EXCLUDE_NONE)
        assert np.array_equal(node_off2, node_off)
        for budget in (24, 1 << 30):
            t.fill_(-1)
            torch.cuda.synchronize(dev)
            assert comm.gather_node_csr(0, 7, budget, o.data_ptr(), t.data_ptr(), r.data_ptr(), E) == E
            assert np.array_equal(t.cpu().numpy(), time2)
            assert np.array_equal(r.cpu().numpy(), rule2 + 7)
    finally:
        eng.set_node_order(_lib.NODE_ORDER_RULE)


def test_no_per_node_result_refused():
    """A ctx whose last per-node call failed (or that has none) refuses the
    gather and the node offsets on every rank (no stale offsets travel)."""
    from cronsun_amd.engine import Comm, Engine
    eng = Engine(0)
    comm = Comm(eng, 1, 0, Comm.unique_id())
    try:
        for call in (lambda: comm.node_offsets(4), lambda: comm.gather_node_csr(0, 0, 1 << 20, 0, 0, 0, 0)):
            with pytest.raises(_lib.CgError) as err:
                call()
            assert err.value.code == _lib.CG_EINVAL
    finally:
        comm.free()
        eng.close()


def test_comm_then_torch_exits_cleanly():
    """RCCL loaded by the library first, torch imported afterwards: one RCCL
    copy in the process and a clean exit (round 4 aborted in the heap check at
    exit, tools/probe_comm_exit.py)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for mode in ("comm_torch", "torch_comm"):
        p = subprocess.run([sys.executable, os.path.join(root, "tools", "probe_comm_exit.py"), mode],
                           capture_output=True, text=True, timeout=150)
        assert p.returncode == 0, (mode, p.returncode, p.stdout[-2000:], p.stderr[-2000:])
        assert f"done {mode}" in p.stdout and "rccl copies 1" in p.stdout, (mode, p.stdout[-2000:])


@pytest.mark.parametrize("world,budget", [(2, 12 * 5000), (3, 1 << 31), (8, 12 * 777), (64, 12 * 40000)])
def test_merge_ranks_random(world, budget):
    """cg_node_csr_merge_ranks (the time-ordered gather's merge, also run by
    cg_comm_gather_node_csr on root): every node's rank runs, each in (time,
    rule) order with rank g's rules below rank g+1's, merged in place into
    (time, rule) order -- a stable sort by time of the node's list.  Many equal
    times (ties across runs), empty runs, nodes with one non-empty run, a node
    larger than the scratch budget, up to 64 ranks."""
    import torch
    rng = np.random.default_rng(world)
    N = 300
    cnt = rng.integers(0, 60, (N, world))
    cnt[rng.random((N, world)) < 0.3] = 0
    cnt[5] = 0
    cnt[6, :] = 0
    cnt[6, world // 2] = 500  # one non-empty run: nothing to merge
    cnt[7] = 2000  # larger than the smallest budgets' groups
    rb = np.zeros((N, world + 1), dtype=np.int64)
    rb[:, 1:] = np.cumsum(cnt, axis=1)
    base = np.concatenate([[0], np.cumsum(rb[:, -1])[:-1]])
    rb += base[:, None]
    E = int(rb[-1, -1])
    t = np.empty(E, dtype=np.int64)
    r = np.empty(E, dtype=np.int32)
    for n in range(N):
        for g in range(world):
            a, b = rb[n, g], rb[n, g + 1]
            tt = np.sort(rng.integers(1767571200, 1767571200 + 40, b - a))
            rr = rng.integers(g * 1000, g * 1000 + 1000, b - a).astype(np.int32)
            o = np.lexsort((rr, tt))
            t[a:b], r[a:b] = tt[o], rr[o]
    exp_t, exp_r = t.copy(), r.copy()
    for n in range(N):
        a, b = rb[n, 0], rb[n, -1]
        o = np.argsort(t[a:b], kind="stable")
        exp_t[a:b], exp_r[a:b] = t[a:b][o], r[a:b][o]
    from cronsun_amd.engine import Engine
    dev = torch.device("cuda", 0)
    dt, dr = torch.from_numpy(t).to(dev), torch.from_numpy(r).to(dev)  # torch first (its own context)
    torch.cuda.synchronize(dev)
    eng = Engine(0)
    try:
        eng.node_csr_merge_ranks(N, world, rb, dt.data_ptr(), dr.data_ptr(), budget)
    finally:
        eng.close()
    assert np.array_equal(dt.cpu().numpy(), exp_t)
    assert np.array_equal(dr.cpu().numpy(), exp_r)


@pytest.mark.parametrize("world", [2, 3])
def test_comm_world2_one_gpu(tmp_path, world):
    """The library's multi-rank exchange for real at world 2 and 3 on one GPU
    (tools/comm_world2.py: each rank claims its own NCCL_HOSTID, so RCCL
    accepts two ranks on one device and moves the data over its socket
    transport): all-gather, node offsets, and cg_comm_gather_node_csr of
    job-ID-range shards in time order (ranks' runs merged on the root by
    k_merge_ranks) and rule order, roots 0 and world - 1, budgets of 24 B per
    rank (every chunk split), a third of the largest node and 1 GiB -- equal
    to the unsharded per-node lists; and time-ordered results whose rule
    bases descend with the rank refused with CG_EINVAL on every rank."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "tools", "comm_world2.py"), str(tmp_path), str(world)],
                       capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-5000:])
    recs = {g: [json.loads(x) for x in open(tmp_path / f"rank{g}.jsonl")] for g in range(world)}
    for g in range(world):
        cases = {}
        for x in recs[g]:
            cases.setdefault(x["case"], []).append(x)
        assert cases["done"]
        assert cases["allgather"][0]["got"] == [[q * 10 + 1, -q] for q in range(world)]
        assert cases["allgather_after"][0]["got"] == [[q] for q in range(world)]
        assert cases["descending_bases"][0]["code"] == cases["descending_bases"][0]["expect"]
        for x in cases.get("node_offsets", []):
            assert x["ok"], x
        for x in cases.get("gather", []):
            assert x["ok"], x
    n_gathers = sum(1 for g in range(world) for x in recs[g] if x["case"] == "gather")
    assert n_gathers == 2 * 3 * len({0, world - 1})


def test_merge_scratch_capped_at_the_merged_events():
    """A small merge with the default 2-GiB budget allocates scratch for its
    own events, not the budget's 179 M (2.1 GB of HBM held until
    close)."""
    import torch
    from cronsun_amd.engine import Engine
    dev = torch.device("cuda", 0)
    N, world = 50, 4
    rng = np.random.default_rng(3)
    cnt = rng.integers(0, 30, (N, world))
    rb = np.zeros((N, world + 1), dtype=np.int64)
    rb[:, 1:] = np.cumsum(cnt, axis=1)
    rb += np.concatenate([[0], np.cumsum(rb[:, -1])[:-1]])[:, None]
    E = int(rb[-1, -1])
    t = np.empty(E, dtype=np.int64)
    r = np.empty(E, dtype=np.int32)
    for n in range(N):
        for g in range(world):
            a, b = rb[n, g], rb[n, g + 1]
            t[a:b] = np.sort(rng.integers(0, 20, b - a)) + 1767571200
            r[a:b] = np.arange(b - a) + 1000 * g
    dt, dr = torch.from_numpy(t).to(dev), torch.from_numpy(r).to(dev)
    torch.cuda.synchronize(dev)
    eng = Engine(0)
    try:
        free0 = torch.cuda.mem_get_info(dev)[0]
        eng.node_csr_merge_ranks(N, world, rb, dt.data_ptr(), dr.data_ptr())  # default 2-GiB budget
        used = free0 - torch.cuda.mem_get_info(dev)[0]
    finally:
        eng.close()
    assert used < (64 << 20), used
    exp_t = t.copy()
    for n in range(N):
        a, b = rb[n, 0], rb[n, -1]
        exp_t[a:b] = np.sort(t[a:b], kind="stable")
    assert np.array_equal(dt.cpu().numpy(), exp_t)


def test_shard_helpers_refuse_an_engine_of_another_device():
    """merge_rank_runs / place_node_slice with an engine whose device is not
    the tensors' raise ValueError before the library sees a foreign pointer."""
    import torch
    from cronsun_amd import shard

    class OtherDevice:
        device = 1
    dev = torch.device("cuda", 0)
    t = torch.zeros(8, dtype=torch.int64, device=dev)
    r = torch.zeros(8, dtype=torch.int32, device=dev)
    rb = np.array([[0, 4, 8]], dtype=np.int64)
    with pytest.raises(ValueError, match="engine on device 1"):
        shard.merge_rank_runs(rb, t, r, engine=OtherDevice())
    off = torch.tensor([0, 8], dtype=torch.int64, device=dev)
    with pytest.raises(ValueError, match="engine on device 1"):
        shard.place_node_slice(off, t, r, 0, torch.zeros(1, dtype=torch.int64, device=dev), t, r,
                               engine=OtherDevice())
