"""BASELINE.json configs 3 and 4 at full size on one MI355X, checked against
the oracle.

Config 3: 1M jobs x 10k nodes (500 groups, GroupIDs / NodeIDs /
ExcludeNodeIDs), config-2 spec mix, one 1-h window -> per-node CSR.  Every
node list of a seeded node sample is compared bit-exact with that node's own
filter over every job (node.go:121-158 -> Job.Cmds, job.go:591-614, restated
by the oracle) composed with the oracle's Next loop (spec.go:55-145); the
node-CSR total must equal sum_r fires(r) x |nodes(r)|.

Config 4: 10M rules x 7 d split into 2/4/8 job-ID ranges balanced by
estimated events (the count pass), every range expanded alone
on a second context: stitched offsets equal the unsharded run's, and each
range's times equal the unsharded range (order-sensitive device checksums
over the same global positions, cg_checksum_device); a seeded sample of rules
is bit-exact against the oracle."""
import os

import numpy as np
import pytest

import oracle_lib as O
from cronsun_amd import _lib, cron, shard, synth

pytestmark = pytest.mark.gpu
DAY = 86400


def host_threads():
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return 8


def oracle_scheds(specs):
    """The oracle's own parser (not the product's masks), deduplicated."""
    memo = {}
    out = []
    for s in specs:
        if s not in memo:
            sc, err = O.parse(s)
            assert err is None, (s, err)
            memo[s] = sc
        out.append(memo[s])
    return O.sched_array(out)


@pytest.fixture(scope="module")
def config3():
    from cronsun_amd.engine import Engine
    eng = Engine(0)
    R = 1_000_000
    specs = synth.spec_mix(R, seed=0x5EED + 3, mix=synth.MIX_CONFIG2)
    arr, status = cron.parse_batch(specs, threads=16)
    assert (status == 0).all()
    rin = synth.rules_for_nodes(R, n_nodes=10_000, n_groups=500, seed=0x5EED + 3)
    t0, t1 = synth.T0_2026, synth.T0_2026 + 3600
    eo, et = O.expand_batch(oracle_scheds(specs), t0, t1, oracle_zone_utc(), threads=host_threads())
    sp = eng.upload_c(arr, R)
    drules = eng.upload_rules(rin)
    yield eng, sp, drules, rin, (t0, t1), (eo, et)
    drules.free()
    sp.free()
    eng.close()


_utc = None


def oracle_zone_utc():
    global _utc
    if _utc is None:
        _utc = O.Loc("UTC")
    return _utc


@pytest.mark.parametrize("mode", [_lib.EXCLUDE_NONE, _lib.EXCLUDE_CUMULATIVE])
def test_config3_full_size_per_node_vs_oracle(config3, mode):
    eng, sp, drules, rin, (t0, t1), (eo, et) = config3
    En, nnz = eng.expand_per_node_rules_device(sp, cron.UTC(), t0, t1, drules, mode)
    node_off = np.empty(rin.n_nodes + 1, dtype=np.int64)
    from cronsun_amd._lib import check, lib
    check(lib().cg_node_result_copy(eng._h, node_off.ctypes.data, None, None, 0))
    assert node_off[0] == 0 and node_off[-1] == En and (np.diff(node_off) >= 0).all()
    # total: every (rule, node) pair carries all of the rule's oracle fires
    rn_off, _ = eng.rule_nodes(rin, mode)
    deg = np.diff(rn_off)
    assert int(rn_off[-1]) == nnz
    assert En == int(np.dot(np.diff(eo), deg)), "node-CSR total != sum fires(r) x |nodes(r)|"
    assert En > 1_000_000_000  # the config-3 scale: ~2.6 G node events per hour
    # bit-exact node lists on a seeded sample of nodes
    nodes = np.sort(np.random.default_rng(100 + mode).choice(rin.n_nodes, 96, replace=False))
    roff, rules = O.node_rules(rin, mode, nodes, threads=host_threads())
    for k, n in enumerate(nodes):
        exp_t, exp_r = O.node_list(eo, et, rules[roff[k]:roff[k + 1]])
        got_t, got_r = eng.node_copy_range(node_off[n], node_off[n + 1] - node_off[n])
        assert np.array_equal(got_r, exp_r), f"node {n}: rule ids differ"
        assert np.array_equal(got_t, exp_t), f"node {n}: fire times differ"


def test_config4_sharded_ranges_stitch_to_unsharded():
    from cronsun_amd.engine import Engine
    total, base_n = 10_000_000, 1_000_000
    t0, t1 = synth.T0_2026, synth.T0_2026 + 7 * DAY
    base_specs = synth.spec_mix(base_n, seed=0x5EED + 4, mix=synth.MIX_LIGHT)
    base_arr, status = cron.parse_batch(base_specs, threads=16)
    assert (status == 0).all()
    # the global 10M-rule set: rule i = base[i % 1M] (bench.py --workload config4)
    tiled = np.ascontiguousarray(np.tile(np.ctypeslib.as_array(base_arr), total // base_n))
    carr = (base_arr._type_ * total).from_buffer(tiled)
    utc = cron.UTC()
    A, B = Engine(0), Engine(0)
    try:
        spA = A.upload_c(carr, total)
        E = A.expand_device(spA, utc, t0, t1)
        offA = np.empty(total + 1, dtype=np.int64)
        from cronsun_amd._lib import check, lib
        check(lib().cg_result_copy_offsets(A._h, offA.ctypes.data))
        assert offA[-1] == E and E > 10_000_000_000
        _, dA, _ = A.result_device()
        spB = B.upload_c(carr, total)
        counts = B.count(spB, utc, t0, t1)  # the count pass of §8e
        assert np.array_equal(counts, np.diff(offA))
        block = 65536
        nb = (total + block - 1) // block
        weights = np.add.reduceat(counts, np.arange(0, total, block)).astype(np.float64) + 1e-9
        for world in (2, 4, 8):
            ranges = []
            for k in range(world):
                c0, c1 = shard.shard_range(nb, world, k, weights=weights)
                ranges.append((c0 * block, min(c1 * block, total)))
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            assert all(ranges[k][1] == ranges[k + 1][0] for k in range(world - 1))
            ev = [int(offA[hi] - offA[lo]) for lo, hi in ranges]
            assert max(ev) <= E / world * 1.02 + counts.max() * block, (world, ev)
            for lo, hi in ranges:
                view = spB.slice(lo, hi - lo)
                Ek = B.expand_device(view, utc, t0, t1)
                assert Ek == offA[hi] - offA[lo], (world, lo, hi)
                offB = np.empty(hi - lo + 1, dtype=np.int64)
                check(lib().cg_result_copy_offsets(B._h, offB.ctypes.data))
                assert np.array_equal(offB + offA[lo], offA[lo:hi + 1]), (world, lo, hi)
                _, dB, _ = B.result_device()
                ckB = B.checksum(dB, Ek, 8, first_index=int(offA[lo]))
                ckA = A.checksum(dA + int(offA[lo]) * 8, Ek, 8, first_index=int(offA[lo]))
                assert ckA == ckB, (world, lo, hi)
                view.free()
        # checksums are additive: the ranges of the last split add up to the whole
        whole = A.checksum(dA, E, 8)
        parts = sum(A.checksum(dA + int(offA[lo]) * 8, int(offA[hi] - offA[lo]), 8,
                               first_index=int(offA[lo])) for lo, hi in ranges) % (1 << 64)
        assert whole == parts
        # bit-exact on a seeded sample of the 10M rules against the oracle
        idx = np.sort(np.random.default_rng(44).choice(total, 3000, replace=False))
        sample = oracle_scheds([base_specs[i % base_n] for i in idx])
        eo, et = O.expand_batch(sample, t0, t1, oracle_zone_utc(), threads=host_threads())
        for k, i in enumerate(idx):
            got = A.copy_times(offA[i], offA[i + 1] - offA[i])
            assert np.array_equal(got, et[eo[k]:eo[k + 1]]), base_specs[i % base_n]
    finally:
        A.close()
        B.close()


@pytest.mark.parametrize("order", ["rule", "time"])
def test_config3_sharded_ranges_place_to_unsharded(config3, order):
    """North_star's second collective on one GPU: config 3 (1M jobs x 10k
    nodes, 1 h) split into 2/4/8 job-ID ranges, every range's per-node CSR
    computed alone on a second context and placed into the gathered per-node
    CSR by the library's kernel (cg_node_csr_place: node n's slice of range g
    at node_base[n] + sum_{g' < g} count[g'][n], rule indices made global),
    exactly as shard.gather_node_csr does on rank 0 after the RCCL transfers.
    The placed CSR must equal the unsharded one (order-sensitive device
    checksums of times and rules), and a node sample is bit-exact against the
    oracle (node.go:121-158 -> Job.Cmds over every job, in job-ID order).
    order "time": every range's lists in (time, rule) order
    (cg_set_node_order(TIME), the byTime order of each node's Cron,
    cron.go:64-79,220), placed and then merged per node by the library
    (cg_node_csr_merge_ranks, what cg_comm_gather_node_csr runs on root):
    equal to the unsharded time-ordered lists."""
    import torch
    from cronsun_amd.engine import Engine
    eng, sp, drules, rin, (t0, t1), (eo, et) = config3
    utc = cron.UTC()
    timed = order == "time"
    if timed:
        eng.set_node_order(_lib.NODE_ORDER_TIME)
    try:
        En, _ = eng.expand_per_node_rules_device(sp, utc, t0, t1, drules, _lib.EXCLUDE_NONE)
    finally:
        eng.set_node_order(_lib.NODE_ORDER_RULE)
    node_off = np.empty(rin.n_nodes + 1, dtype=np.int64)
    from cronsun_amd._lib import check, lib
    check(lib().cg_node_result_copy(eng._h, node_off.ctypes.data, None, None, 0))
    _, dt, dr, _ = eng.node_result_device()
    ck_t, ck_r = eng.checksum(dt, En, 8), eng.checksum(dr, En, 4)
    dev = torch.device("cuda", 0)
    N, R = rin.n_nodes, rin.n_rules
    B = Engine(0)
    if timed:
        B.set_node_order(_lib.NODE_ORDER_TIME)
    try:
        arr, _ = cron.parse_batch(synth.spec_mix(R, seed=0x5EED + 3, mix=synth.MIX_CONFIG2), threads=16)
        spB = B.upload_c(arr, R)
        out_t = torch.empty(En, dtype=torch.int64, device=dev)
        out_r = torch.empty(En, dtype=torch.int32, device=dev)
        for world in (2, 4, 8):
            ranges = [shard.shard_range(R, world, g) for g in range(world)]
            parts = []
            for lo, hi in ranges:
                view = spB.slice(lo, hi - lo)
                dr_g = B.upload_rules(rin.slice_rules(lo, hi))
                parts.append((view, dr_g))
            allc = torch.zeros(world, N, dtype=torch.int64, device=dev)
            for g, (view, dr_g) in enumerate(parts):  # the per-node counts every rank all-gathers
                B.expand_per_node_rules_device(view, utc, t0, t1, dr_g, _lib.EXCLUDE_NONE)
                B.node_counts_to_device(allc[g].data_ptr())
            assert int(allc.sum()) == En
            out_t.fill_(-1)
            allc_h = allc.cpu().numpy()
            for g, ((lo, hi), (view, dr_g)) in enumerate(zip(ranges, parts)):
                B.expand_per_node_rules_device(view, utc, t0, t1, dr_g, _lib.EXCLUDE_NONE)
                n_off, n_time, n_rule = B.node_result_tensors(N)  # zero-copy views of B's result
                starts, node_base = shard.node_slice_starts(allc, g)
                # the product path of shard.gather_node_csr: torch's stream synchronised, then the kernel
                shard.place_node_slice(n_off, n_time, n_rule, lo, starts, out_t, out_r, engine=B)
                view.free()
                dr_g.free()
            torch.cuda.synchronize(dev)
            if timed:
                # run g of node n: [node_base[n] + sum_{g' < g} count[g'][n], ...)
                rb = np.empty((N, world + 1), dtype=np.int64)
                rb[:, 0] = node_off[:-1]
                rb[:, 1:] = node_off[:-1, None] + np.cumsum(allc_h.T, axis=1)
                assert np.array_equal(rb[:, world], node_off[1:])
                # a small budget: many node groups through the scratch copy
                shard.merge_rank_runs(rb, out_t, out_r, engine=B, budget_bytes=12 << 24)
            assert np.array_equal(node_base.cpu().numpy(), node_off), world
            assert B.checksum(out_t.data_ptr(), En, 8) == ck_t, world
            assert B.checksum(out_r.data_ptr(), En, 4) == ck_r, world
        nodes = np.sort(np.random.default_rng(303).choice(N, 24, replace=False))
        roff, rules = O.node_rules(rin, _lib.EXCLUDE_NONE, nodes, threads=host_threads())
        for k, n in enumerate(nodes):
            exp_t, exp_r = O.node_list(eo, et, rules[roff[k]:roff[k + 1]])
            if timed:  # (time, rule): the rule-major list sorted stably by time
                o = np.argsort(exp_t, kind="stable")
                exp_t, exp_r = exp_t[o], exp_r[o]
            a, b = int(node_off[n]), int(node_off[n + 1])
            assert np.array_equal(out_r[a:b].cpu().numpy(), exp_r), n
            assert np.array_equal(out_t[a:b].cpu().numpy(), exp_t), n
    finally:
        B.close()
