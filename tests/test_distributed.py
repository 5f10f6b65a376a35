"""The N > 1 path on CPU: job-ID-range sharding and the two small collectives
(global CSR offsets, per-node offsets) with torch.distributed over gloo,
world_size 2.  Expansion itself is the oracle here (no GPU on this host);
the check is that sharded + stitched output equals the unsharded one."""
import os
import socket

import numpy as np
import pytest

import oracle_lib as O
from cronsun_amd import shard

DAY = 86400
T0 = 1767571200


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _specs():
    from cronsun_amd import synth
    return synth.spec_mix(600, seed=17)


def _worker(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    specs = _specs()
    lo, hi = shard.shard_range(len(specs), world, rank)
    arr = O.sched_array([O.parse(s)[0] for s in specs[lo:hi]])
    off, times = O.expand_batch(arr, T0, T0 + DAY, O.Loc("UTC"), threads=2)
    base, total, per_rank = shard.global_offsets(int(off[-1]), dist)
    # per-node: node n gets rule r iff r % 7 == n % 7 (a toy rule->node map)
    N = 7
    counts = torch.zeros(N, dtype=torch.int64)
    for k, r in enumerate(range(lo, hi)):
        counts[r % N] += int(off[k + 1] - off[k])
    my_off, node_base = shard.node_offsets(counts, dist)
    g = shard.gather_csr(torch.from_numpy(off.astype(np.int64)), torch.from_numpy(times.astype(np.int64)),
                         dist)
    extra = {} if g is None else {"g_off": g[0].numpy(), "g_times": g[1].numpy()}
    np.savez(os.path.join(outdir, f"r{rank}.npz"), off=off, times=times, base=base, total=total,
             lo=lo, hi=hi, my_off=my_off.numpy(), node_base=node_base.numpy(), **extra)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    for n in (0, 1, 7, 1000):
        for w in (1, 2, 3, 8):
            rs = [shard.shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
    wts = np.array([1] * 50 + [100] * 10 + [1] * 40)
    rs = [shard.shard_range(100, 4, r, weights=wts) for r in range(4)]
    assert rs[0][0] == 0 and rs[-1][1] == 100 and all(a <= b for a, b in rs)


def test_two_rank_gloo_stitch(tmp_path):
    import torch.multiprocessing as mp
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = np.load(tmp_path / "r0.npz")
    r1 = np.load(tmp_path / "r1.npz")
    specs = _specs()
    arr = O.sched_array([O.parse(s)[0] for s in specs])
    off, times = O.expand_batch(arr, T0, T0 + DAY, O.Loc("UTC"), threads=4)
    assert int(r0["base"]) == 0 and int(r1["base"]) == int(r0["off"][-1])
    assert int(r0["total"]) == int(r1["total"]) == int(off[-1])
    stitched = np.concatenate([r0["times"], r1["times"]])
    assert np.array_equal(stitched, times)
    stitched_off = np.concatenate([r0["off"][:-1], r1["off"] + r0["off"][-1]])
    assert np.array_equal(stitched_off, off)
    # the optional CSR gather to rank 0 (grouped point-to-point)
    assert np.array_equal(r0["g_off"], off) and np.array_equal(r0["g_times"], times)
    assert "g_off" not in r1
    # per-node offsets: rank 1's slice of node n starts after rank 0's
    N = 7
    cnt = np.zeros(N, dtype=np.int64)
    for r in range(len(specs)):
        cnt[r % N] += off[r + 1] - off[r]
    assert np.array_equal(r0["node_base"], np.concatenate([[0], np.cumsum(cnt)]))
    c0 = np.zeros(N, dtype=np.int64)
    for r in range(int(r0["lo"]), int(r0["hi"])):
        c0[r % N] += off[r + 1] - off[r]
    assert np.array_equal(r0["my_off"], r0["node_base"][:-1])
    assert np.array_equal(r1["my_off"], r0["node_base"][:-1] + c0)


def _skewed_specs():
    # the first fifth of the job-ID order fires every few seconds, the rest hourly
    return ["*/3 * * * * *"] * 120 + ["0 0 * * * *"] * 480


def _balance_worker(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    specs = _skewed_specs()

    def count_fn(lo, hi):  # the oracle stands in for Engine.count (no GPU here)
        arr = O.sched_array([O.parse(s)[0] for s in specs[lo:hi]])
        off, _ = O.expand_batch(arr, T0, T0 + DAY, O.Loc("UTC"), threads=2, with_times=False)
        return np.diff(off)

    lo, hi, w = shard.event_balanced_range(len(specs), count_fn, dist, block=16)
    np.savez(os.path.join(outdir, f"b{rank}.npz"), lo=lo, hi=hi, w=w)
    dist.barrier()
    dist.destroy_process_group()


def test_event_balanced_ranges_gloo(tmp_path):
    """§8e: ranges balanced by estimated events (count pass + one all-gather
    of per-block sums), contiguous in job-ID order, identical on every rank."""
    import torch.multiprocessing as mp
    world = 3
    mp.spawn(_balance_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rs = [np.load(tmp_path / f"b{r}.npz") for r in range(world)]
    specs = _skewed_specs()
    cuts = [(int(x["lo"]), int(x["hi"])) for x in rs]
    assert cuts[0][0] == 0 and cuts[-1][1] == len(specs)
    assert all(cuts[i][1] == cuts[i + 1][0] for i in range(world - 1))
    assert all(np.array_equal(rs[0]["w"], x["w"]) for x in rs)
    arr = O.sched_array([O.parse(s)[0] for s in specs])
    off, _ = O.expand_batch(arr, T0, T0 + DAY, O.Loc("UTC"), threads=2, with_times=False)
    ev = [int(off[hi] - off[lo]) for lo, hi in cuts]
    # an equal rule split would put nearly all events on rank 0 ([3.45M, 11K, 11K]);
    # balanced to within a block (16 rules x 28800 fires) per cut
    assert max(ev) - min(ev) <= 2 * 16 * 28800, ev
    assert min(ev) > 0.5 * max(ev), ev
    assert int(rs[0]["w"].sum()) == int(off[-1])


def _node_csr_oracle(rin, mode, specs, t0, t1):
    """Per-node (time, rule) CSR of a rule set from the oracle: every node's
    own filter over all rules (node.go:121-158 -> Job.Cmds) composed with the
    Next loop; rules ascending within a node."""
    arr = O.sched_array([O.parse(s)[0] for s in specs])
    eo, et = O.expand_batch(arr, t0, t1, O.Loc("UTC"), threads=2)
    roff, rules = O.node_rules(rin, mode, np.arange(rin.n_nodes), threads=2)
    node_off = [0]
    ts, rs = [], []
    for n in range(rin.n_nodes):
        t, r = O.node_list(eo, et, rules[roff[n]:roff[n + 1]])
        ts.append(t)
        rs.append(r)
        node_off.append(node_off[-1] + len(t))
    return (np.array(node_off, dtype=np.int64), np.concatenate(ts).astype(np.int64),
            np.concatenate(rs).astype(np.int32))


def _gather_worker(rank, world, port, outdir, mode, budget, order="rule"):
    import torch
    import torch.distributed as dist
    from cronsun_amd import synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rin = synth.multi_rule_jobs(160, seed=5, key_choices=2)
    specs = synth.spec_mix(rin.n_rules, seed=6, mix=synth.MIX_LIGHT)
    # job-ID-range shards: cut at the job boundaries nearest to equal rule counts
    starts = np.concatenate([[0], np.nonzero(np.diff(rin.rule_job))[0] + 1, [rin.n_rules]])
    cuts = [int(starts[np.argmin(np.abs(starts - rin.n_rules * g // world))]) for g in range(world)]
    cuts.append(rin.n_rules)
    lo, hi = cuts[rank], cuts[rank + 1]
    part = rin.slice_rules(lo, hi)
    off, t, r = _node_csr_oracle(part, mode, specs[lo:hi], T0, T0 + DAY)
    if order == "time":  # this rank's lists in (time, rule) order, as cg_set_node_order(TIME) leaves them
        t, r = _time_order(off, t, r)
    g = shard.gather_node_csr(torch.from_numpy(off), torch.from_numpy(t), torch.from_numpy(r), lo, dist,
                              budget_bytes=budget, order=order)
    cnt = torch.from_numpy(np.diff(off))
    allc = torch.zeros(world * rin.n_nodes, dtype=torch.int64)
    dist.all_gather_into_tensor(allc, cnt)
    plan = shard.node_gather_plan(allc.view(world, -1).numpy(), 0, budget)
    if g is not None:
        np.savez(os.path.join(outdir, f"g{rank}.npz"), node_off=g[0].numpy(), time=g[1].numpy(),
                 rule=g[2].numpy(), plan=np.array(plan, dtype=np.int64).reshape(-1, 4))
    dist.barrier()
    dist.destroy_process_group()


def _time_order(node_off, t, r):
    """Every node's list of a rule-major per-node CSR in (time, rule) order."""
    t, r = t.copy(), r.copy()
    for n in range(len(node_off) - 1):
        a, b = int(node_off[n]), int(node_off[n + 1])
        o = np.lexsort((r[a:b], t[a:b]))
        t[a:b], r[a:b] = t[a:b][o], r[a:b][o]
    return t, r


@pytest.mark.parametrize("mode,budget", [(0, shard.DEFAULT_GATHER_BUDGET), (2, shard.DEFAULT_GATHER_BUDGET),
                                         (0, 12 * 700), (1, 12 * 3000)])
def test_gather_node_csr_gloo(tmp_path, mode, budget):
    """north_star's per-node CSR gather: job-ID-range shards, each with its
    own per-node lists, gathered on rank 0 into exactly the per-node CSR of the
    unsharded rule set (world_size 3, three exclude modes; Rule.IDs repeat
    inside jobs, so Job.Cmds' key drops rules).  Small budgets force the
    chunked transfer: several node-range chunks and nodes split into parts."""
    import torch.multiprocessing as mp
    from cronsun_amd import synth
    world = 3
    mp.spawn(_gather_worker, args=(world, _free_port(), str(tmp_path), mode, budget), nprocs=world, join=True)
    got = np.load(tmp_path / "g0.npz")
    assert not (tmp_path / "g1.npz").exists()
    plan = got["plan"]
    if budget < shard.DEFAULT_GATHER_BUDGET:
        assert len(plan) >= 3 and (plan[:, 3] > 1).any() and (plan[:, 3] == 1).any(), plan
    else:
        assert len(plan) == 1
    rin = synth.multi_rule_jobs(160, seed=5, key_choices=2)
    specs = synth.spec_mix(rin.n_rules, seed=6, mix=synth.MIX_LIGHT)
    exp = _node_csr_oracle(rin, mode, specs, T0, T0 + DAY)
    assert np.array_equal(got["node_off"], exp[0])
    assert np.array_equal(got["time"], exp[1])
    assert np.array_equal(got["rule"], exp[2])


@pytest.mark.parametrize("world,dst", [(2, 0), (3, 1), (8, 0)])
def test_node_gather_plan_covers_every_event_within_budget(world, dst):
    """The chunk plan (shared by shard.gather_node_csr and the library's
    cg_comm_gather_node_csr): every peer event is in exactly one piece, pieces
    of a rank are contiguous and in order, and no chunk exceeds the budget."""
    rng = np.random.default_rng(world)
    N = 500
    allc = rng.integers(0, 40, (world, N))
    allc[:, rng.integers(0, N, 5)] = rng.integers(500, 3000, (world, 5))  # a few big nodes
    for budget in (12 * 2 * world, 12 * 97, 12 * 1000, 12 * 10**9):
        plan = shard.node_gather_plan(allc, dst, budget)
        offs = np.zeros((world, N + 1), dtype=np.int64)
        offs[:, 1:] = np.cumsum(allc, axis=1)
        nxt = [0] * world
        for ch in plan:
            tot = 0
            for g in range(world):
                if g == dst:
                    continue
                lo, hi = shard._piece(offs[g], allc[g], ch)
                if hi > lo:
                    assert lo == nxt[g], (budget, ch, g)
                    nxt[g] = hi
                tot += hi - lo
            assert 0 < tot * 12 <= budget, (budget, ch)
        assert all(nxt[g] == offs[g, -1] for g in range(world) if g != dst)


@pytest.mark.parametrize("world,budget", [(3, shard.DEFAULT_GATHER_BUDGET), (3, 12 * 700), (2, 12 * 3000)])
def test_gather_node_csr_time_ordered_gloo(tmp_path, world, budget):
    """Time-ordered per-node lists at N > 1 (the byTime order of every node's
    Cron, cron.go:64-79,220): each rank's lists in (time, rule) order, gathered
    on rank 0 and merged per node by (time, global rule) -- equal to the
    unsharded lists in (time, rule) order.  Concatenating the ranks' slices
    (order="rule") would not be."""
    import torch.multiprocessing as mp
    from cronsun_amd import synth
    mp.spawn(_gather_worker, args=(world, _free_port(), str(tmp_path), 0, budget, "time"), nprocs=world, join=True)
    got = np.load(tmp_path / "g0.npz")
    rin = synth.multi_rule_jobs(160, seed=5, key_choices=2)
    specs = synth.spec_mix(rin.n_rules, seed=6, mix=synth.MIX_LIGHT)
    exp_off, exp_t, exp_r = _node_csr_oracle(rin, 0, specs, T0, T0 + DAY)
    exp_t, exp_r = _time_order(exp_off, exp_t, exp_r)
    assert np.array_equal(got["node_off"], exp_off)
    assert np.array_equal(got["time"], exp_t)
    assert np.array_equal(got["rule"], exp_r)


def _bases_worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off = torch.tensor([0, 2, 3], dtype=torch.int64)
    t = torch.tensor([T0 + 1, T0 + 2, T0 + 1], dtype=torch.int64)
    r = torch.tensor([0, 1, 0], dtype=torch.int32)
    for order in ("time", "rule"):
        # rank 1's range before rank 0's: ties merged by rank would be out of
        # (time, global rule) order, so the time-ordered gather refuses on every
        # rank; the rule-ordered gather needs no rank order and runs
        try:
            shard.gather_node_csr(off, t, r, 1000 * (world - rank), dist, order=order)
            res = "ok"
        except ValueError as e:
            res = str(e)
        with open(os.path.join(outdir, f"{order}{rank}.txt"), "w") as f:
            f.write(res)
    dist.barrier()
    dist.destroy_process_group()


def test_time_ordered_gather_refuses_descending_rule_bases(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_bases_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for g in range(world):
        assert "does not ascend" in (tmp_path / f"time{g}.txt").read_text()
        assert (tmp_path / f"rule{g}.txt").read_text() == "ok"


def test_gather_node_csr_requires_order():
    """The Python gather cannot tell the lists' order: the caller states it."""
    with pytest.raises(TypeError):
        shard.gather_node_csr(None, None, None, 0, None)
    with pytest.raises(ValueError):
        import torch
        z = torch.zeros(1, dtype=torch.int64)
        shard.gather_node_csr(z, z, z.to(torch.int32), 0, None, order="byTime")


@pytest.mark.parametrize("world,dst", [(2, 0), (3, 1), (8, 0), (8, 5)])
def test_library_gather_plan_equals_python(world, dst):
    """The library's chunk plan (cg_comm_gather_plan: the plan
    cg_comm_gather_node_csr executes over RCCL) equals shard.node_gather_plan
    chunk for chunk at worlds 2/3/8, including split nodes and tiny budgets,
    and rejects a budget below 24 bytes per rank as the Python plan does."""
    from cronsun_amd import _lib
    from cronsun_amd.engine import comm_gather_plan
    rng = np.random.default_rng(100 + world + dst)
    N = 700
    allc = rng.integers(0, 40, (world, N))
    allc[:, rng.integers(0, N, 7)] = rng.integers(500, 3000, (world, 7))
    allc[:, rng.integers(0, N, 50)] = 0
    for budget in (12 * 2 * world, 12 * 97, 12 * 1000, 12 * 5000, 12 * 10**9):
        assert comm_gather_plan(allc, dst, budget) == shard.node_gather_plan(allc, dst, budget), budget
    with pytest.raises(_lib.CgError):
        comm_gather_plan(allc, dst, 12 * 2 * world - 12)
    with pytest.raises(ValueError):
        shard.node_gather_plan(allc, dst, 12 * 2 * world - 12)
