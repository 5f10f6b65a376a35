"""BASELINE config 3 over its whole 24-h horizon on one MI355X: 1M jobs x 10k
nodes (500 groups, GroupIDs / NodeIDs / ExcludeNodeIDs), config-2 spec mix,
24 consecutive one-hour windows through the pipelined per-node entry point
(cg_expand_per_node_rules_device_async + cg_expand_per_node_wait; a node's
scheduler filtering every job, node/node.go:121-158, and firing its Cron
entries hour after hour, cron.go:210-275).  Every window's lists of a seeded
sample of 48 nodes are compared bit-exact with the oracle, in rule order
(Job.Cmds' evaluation order, job.go:591-614) and in (time, rule) order
(cg_set_node_order(TIME): Cron.run's sort.Sort(byTime), cron.go:64-79,220).

The oracle expands the sampled nodes' rules window by window (spec.go:55-145,
constantdelay.go:25-27 restated): each window is the Next loop started at the
window's own start, which for @every rules (Next(t) = t + D) differs from a
slice of one day-long loop."""
import numpy as np
import pytest

import oracle_lib as O
from cronsun_amd import _lib, cron, synth
from test_gpu_configs import host_threads, oracle_scheds, oracle_zone_utc

pytestmark = pytest.mark.gpu
HOUR = 3600


@pytest.fixture(scope="module")
def day():
    from cronsun_amd.engine import Engine
    eng = Engine(0)
    R = 1_000_000
    specs = synth.spec_mix(R, seed=0x5EED + 3, mix=synth.MIX_CONFIG2)
    arr, status = cron.parse_batch(specs, threads=16)
    assert (status == 0).all()
    rin = synth.rules_for_nodes(R, n_nodes=10_000, n_groups=500, seed=0x5EED + 3)
    t0 = synth.T0_2026
    nodes = np.sort(np.random.default_rng(2404).choice(rin.n_nodes, 48, replace=False))
    roff, nrules = O.node_rules(rin, _lib.EXCLUDE_NONE, nodes, threads=host_threads())
    uniq = np.unique(nrules)
    osch = oracle_scheds([specs[r] for r in uniq])
    sp = eng.upload_c(arr, R)
    dr = eng.upload_rules(rin)
    yield eng, sp, dr, rin, t0, nodes, roff, nrules, uniq, osch
    dr.free()
    sp.free()
    eng.close()


def expected_window(eo, et, uniq, rules):
    """One node's rule-major list from the oracle's window expansion of uniq."""
    return O.node_list(eo, et, np.searchsorted(uniq, rules))


@pytest.mark.parametrize("order", ["rule", "time"])
def test_config3_every_window_of_the_day(day, order):
    eng, sp, dr, rin, t0, nodes, roff, nrules, uniq, osch = day
    from cronsun_amd._lib import check, lib
    utc = cron.UTC()
    try:
        # sizes the outputs (and caches the join): a two-hour window holds
        # more than any one hour
        E2, _ = eng.expand_per_node_rules_device(sp, utc, t0, t0 + 2 * HOUR, dr, _lib.EXCLUDE_NONE)
        assert E2 > 2_000_000_000
        eng.set_node_order(_lib.NODE_ORDER_TIME if order == "time" else _lib.NODE_ORDER_RULE)
        off = np.empty(rin.n_nodes + 1, np.int64)
        total = 0
        for w in range(24):
            a, b = t0 + w * HOUR, t0 + (w + 1) * HOUR
            eng.expand_per_node_async(sp, utc, a, b, dr, _lib.EXCLUDE_NONE)
            En = eng.expand_per_node_wait()
            total += En
            check(lib().cg_node_result_copy(eng._h, off.ctypes.data, None, None, 0))
            assert off[-1] == En
            eo, et = O.expand_batch(osch, a, b, oracle_zone_utc(), threads=host_threads())
            for k, n in enumerate(nodes):
                rules = nrules[roff[k]:roff[k + 1]]
                exp_t, exp_p = expected_window(eo, et, uniq, rules)
                exp_r = uniq[exp_p].astype(np.int32)
                if order == "time":  # rule-major input: a stable sort by time gives (time, rule)
                    o = np.argsort((exp_t - a).astype(np.uint16), kind="stable")
                    exp_t, exp_r = exp_t[o], exp_r[o]
                got_t, got_r = eng.node_copy_range(off[n], off[n + 1] - off[n])
                assert len(got_t) == len(exp_t), (w, n)
                assert np.array_equal(got_t, exp_t), (w, n, "times")
                assert np.array_equal(got_r, exp_r), (w, n, "rules")
        assert total > 24 * 1_000_000_000
    finally:
        eng.set_node_order(_lib.NODE_ORDER_RULE)
