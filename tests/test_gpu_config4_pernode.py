"""Row n2, north_star's target: "bit-exact per-node fire schedules for 10M
rules x 7-day horizon" (BASELINE.json config 4 with config 3's node model).

One rank's share at N = 8: 1.25M rules of config 4's 10M-rule set (the
1M-rule light-mix block tiled in job-ID order, bench.py --workload config4)
over 10k nodes / 500 groups (synth.rules_for_nodes of the whole 10M-job set,
sliced to the rank's job-ID range, as bench.py --per-node does).  The local
rule indices pass 2^20, so the time-ordered lists take the unpacked path
(16-bit offsets + int32 rules).  One-hour windows spread over the 7 days and
one 30-min window (the bench's), in rule order and in (time, rule) order: every window's node-event total equals
sum_r fires(r) x |nodes(r)| (oracle fire counts, the GPU join's degrees) and
48 seeded nodes' lists are bit-exact against each node's own filter over the
rank's jobs (node/node.go:121-158 -> Job.Cmds, job.go:591-614) composed with
the oracle's Next loop (spec.go:55-145)."""
import numpy as np
import pytest

import oracle_lib as O
from cronsun_amd import _lib, cron, shard, synth
from test_gpu_configs import host_threads, oracle_scheds, oracle_zone_utc

pytestmark = pytest.mark.gpu
DAY = 86400


@pytest.fixture(scope="module")
def share():
    from cronsun_amd.engine import Engine
    total, base_n = 10_000_000, 1_000_000
    lo, hi = shard.shard_range(total, 8, 3)  # rank 3 of 8: rules 3.75M..5M (the tiled block wraps inside)
    R = hi - lo
    base_specs = synth.spec_mix(base_n, seed=0x5EED + 4, mix=synth.MIX_LIGHT)
    base_arr, status = cron.parse_batch(base_specs, threads=16)
    assert (status == 0).all()
    base_np = np.ctypeslib.as_array(base_arr)
    idx = np.arange(lo, hi) % base_n
    a = np.ascontiguousarray(base_np[idx])
    rin = synth.rules_for_nodes(total, n_nodes=10_000, n_groups=500, seed=0x5EED + 4).slice_rules(lo, hi)
    eng = Engine(0)
    sp = eng.upload_c((base_arr._type_ * R).from_buffer(a), R)
    drules = eng.upload_rules(rin)
    specs = [base_specs[i] for i in idx]
    yield eng, sp, drules, rin, specs
    drules.free()
    sp.free()
    eng.close()


def _windows():
    t0 = synth.T0_2026
    hours = [0, 29, 58, 87, 116, 145, 167]  # spread over the 7 days, the last hour included
    # and one 30-min window as bench.py --per-node runs them (32-s time-order slabs)
    return [(t0 + 3600 * h, t0 + 3600 * (h + 1)) for h in hours] + [(t0 + 3600 * 100 + 1800, t0 + 3600 * 101)]


def test_config4_per_node_rank_share(share):
    eng, sp, drules, rin, specs = share
    R = rin.n_rules
    assert R == 1_250_000 and R > (1 << 20)
    utc = cron.UTC()
    osch_all = oracle_scheds(specs)
    nodes = np.sort(np.random.default_rng(0x5EED + 48).choice(rin.n_nodes, 48, replace=False))
    roff, rules = O.node_rules(rin, _lib.EXCLUDE_NONE, nodes, threads=host_threads())
    union = np.unique(rules)
    osch_u = oracle_scheds([specs[int(r)] for r in union])
    rn_off, _ = eng.rule_nodes(rin, _lib.EXCLUDE_NONE)
    deg = np.diff(rn_off)
    checked = 0
    for a, b in _windows():
        counts, _ = O.expand_batch(osch_all, a, b, oracle_zone_utc(), threads=host_threads(), with_times=False)
        total = int(np.dot(np.diff(counts), deg))
        eo, et = O.expand_batch(osch_u, a, b, oracle_zone_utc(), threads=host_threads())
        for order in (_lib.NODE_ORDER_RULE, _lib.NODE_ORDER_TIME):
            eng.set_node_order(order)
            try:
                En, nnz = eng.expand_per_node_rules_device(sp, utc, a, b, drules, _lib.EXCLUDE_NONE)
            finally:
                eng.set_node_order(_lib.NODE_ORDER_RULE)
            assert nnz == int(rn_off[-1])
            assert En == total, (a, order, En, total)
            node_off = np.empty(rin.n_nodes + 1, dtype=np.int64)
            _lib.check(_lib.lib().cg_node_result_copy(eng._h, node_off.ctypes.data, None, None, 0))
            assert node_off[-1] == En and (np.diff(node_off) >= 0).all()
            for k, n in enumerate(nodes):
                pos = np.searchsorted(union, rules[roff[k]:roff[k + 1]])
                exp_t, exp_p = O.node_list(eo, et, pos)
                exp_r = union[exp_p].astype(np.int32)
                if order == _lib.NODE_ORDER_TIME:  # rule-major input: stable by time = (time, rule)
                    o = np.argsort(exp_t, kind="stable")
                    exp_t, exp_r = exp_t[o], exp_r[o]
                got_t, got_r = eng.node_copy_range(node_off[n], node_off[n + 1] - node_off[n])
                assert np.array_equal(got_r, exp_r), (a, order, n)
                assert np.array_equal(got_t, exp_t), (a, order, n)
                checked += len(exp_t)
    assert checked > 1_000_000
