"""Rule -> node resolution and per-node fire lists on the GPU vs the oracle's
restatement of Job.Cmds / GetJobNodes (job.go:591-630, web/job.go:222-257)."""
import numpy as np
import pytest

import oracle_lib as O
from common import oracle_parse_all, oracle_zone, product_zone
from cronsun_amd import _lib, cron, synth

pytestmark = pytest.mark.gpu
DAY = 86400


@pytest.fixture(scope="module")
def eng():
    from cronsun_amd.engine import Engine
    return Engine(0)


def oracle_jobset(rin):
    return O.jobset(rin)


def oracle_rule_nodes(rin, mode):
    js = oracle_jobset(rin)
    L = O.lib()
    out = []
    for r in range(rin.n_rules):
        cand = set(rin.nids[rin.nid_off[r]:rin.nid_off[r + 1]].tolist())
        for g in rin.gids[rin.gid_off[r]:rin.gid_off[r + 1]].tolist():
            cand |= set(rin.group_nodes[rin.group_off[g]:rin.group_off[g + 1]].tolist())
        out.append(sorted(n for n in cand if L.or_rule_on_node(js, mode, r, n)))
    return out


@pytest.mark.parametrize("keys,per", [(0, (1, 4)), (2, (1, 4)), (1, (6, 12))])
@pytest.mark.parametrize("mode", [_lib.EXCLUDE_NONE, _lib.EXCLUDE_RULE, _lib.EXCLUDE_CUMULATIVE])
def test_rule_nodes_vs_oracle(eng, mode, keys, per):
    """keys 2: Rule.IDs drawn from two values, so a job's rules repeat Cmd keys
    and the join drops a rule on the nodes a later same-key rule takes
    (job.go:604-609); keys 1 with 6-12 rules per job: chains of up to 12
    rules of one key (k_rule_nodes sweeps each chain from its last rule)."""
    rin = synth.multi_rule_jobs(400, rules_per_job=per, seed=11 + mode, key_choices=keys)
    off, nodes = eng.rule_nodes(rin, mode)
    exp = oracle_rule_nodes(rin, mode)
    for r in range(rin.n_rules):
        assert nodes[off[r]:off[r + 1]].tolist() == exp[r], (mode, r)


@pytest.mark.parametrize("mode", [_lib.EXCLUDE_NONE, _lib.EXCLUDE_CUMULATIVE])
@pytest.mark.parametrize("zone", ["UTC", "America/New_York"])
def test_per_node_fire_lists_vs_oracle(eng, mode, zone):
    rin = synth.multi_rule_jobs(300, seed=21)
    specs = synth.spec_mix(rin.n_rules, seed=4, mix=synth.MIX_LIGHT)
    scheds = [cron.Parse(s) for s in specs]
    t0, t1 = synth.T0_2026 + 64 * DAY, synth.T0_2026 + 65 * DAY + 3600
    if zone == "America/New_York":
        t0, t1 = 1772953200 - 12 * 3600, 1772953200 + 12 * 3600
    node_off, time, rule = eng.expand_per_node(scheds, product_zone(zone), t0, t1, rin, mode)
    # oracle: per rule fire times, per rule node set, then node-major lists
    arr = O.sched_array(oracle_parse_all(specs))  # the oracle's own parser
    eo, et = O.expand_batch(arr, t0, t1, oracle_zone(zone))
    rn = oracle_rule_nodes(rin, mode)
    per_node = [[] for _ in range(rin.n_nodes)]
    for r in range(rin.n_rules):
        for n in rn[r]:
            per_node[n].append(r)
    for n in range(rin.n_nodes):
        exp_t = np.concatenate([et[eo[r]:eo[r + 1]] for r in per_node[n]] or [np.zeros(0, np.int64)])
        exp_r = np.concatenate([np.full(eo[r + 1] - eo[r], r, np.int32) for r in per_node[n]]
                               or [np.zeros(0, np.int32)])
        got_t = time[node_off[n]:node_off[n + 1]]
        got_r = rule[node_off[n]:node_off[n + 1]]
        assert np.array_equal(got_t, exp_t), n
        assert np.array_equal(got_r, exp_r), n


def _string_world(seed, n_jobs=250, n_nodes=40, n_groups=8):
    """Jobs with string IDs whose Rule.IDs repeat inside a job (including ""
    and " "), interned by the C++ host layer (cg_jobset)."""
    from cronsun_amd.model import Group, Job, JobRule, JobSet
    rng = np.random.default_rng(seed)
    nodes = [f"node-{i}" for i in range(n_nodes)]
    groups = {f"g{g}": Group(f"g{g}", "", list(rng.choice(nodes, int(rng.integers(1, 12)), replace=False)))
              for g in range(n_groups)}
    specs = synth.spec_mix(n_jobs * 4, seed=seed, mix=synth.MIX_CONFIG2)
    jobs, k = [], 0
    for j in range(n_jobs):
        rules = []
        for _ in range(int(rng.integers(1, 5))):
            rid = ["", " ", "a", "b"][int(rng.integers(0, 4))]
            gids = [f"g{rng.integers(0, n_groups + 1)}" for _ in range(rng.integers(0, 3))]
            nids = list(rng.choice(nodes, int(rng.integers(0, 4)), replace=False))
            ex = list(rng.choice(nodes, int(rng.integers(0, 3)), replace=False))
            rules.append(JobRule(rid, specs[k], gids, nids, ex))
            k += 1
        jobs.append(Job(f"job{j}", Rules=rules, Pause=bool(rng.random() < 0.05)))
    return JobSet(jobs, groups), nodes


@pytest.mark.parametrize("order", ["rule", "time"])
@pytest.mark.parametrize("mode", [_lib.EXCLUDE_NONE, _lib.EXCLUDE_RULE, _lib.EXCLUDE_CUMULATIVE])
def test_cmd_keys_per_node_vs_oracle_and_cmds(eng, mode, order):
    """Job.Cmds keeps one Cmd per Job.ID+Rule.ID, the last included rule
    (job.go:604-609; the node's Cron replaces entries by that ID,
    node/node.go:209-211, cron.go:131-135).  Jobs whose rules repeat IDs
    (empty and blank IDs included): every node's list, rule-ordered and
    time-ordered, equals the oracle's; in mode NONE each node's rule set is
    also the union of the host cg_jobset_cmds over the jobs."""
    js, nodes = _string_world(61 + mode)
    rin = js.rules_in()
    assert rin.rule_key is not None
    scheds = js.schedules()
    t0, t1 = synth.T0_2026 + 40 * DAY + 600, synth.T0_2026 + 40 * DAY + 600 + 3600
    if order == "time":
        eng.set_node_order(_lib.NODE_ORDER_TIME)
    try:
        node_off, time, rule = eng.expand_per_node(scheds, None, t0, t1, rin, mode)
    finally:
        eng.set_node_order(_lib.NODE_ORDER_RULE)
    specs = [r.Timer for r in js.rules]
    eo, et = O.expand_batch(O.sched_array(oracle_parse_all(specs)), t0, t1, oracle_zone("UTC"))
    rn = oracle_rule_nodes(rin, mode)
    per_node = [[] for _ in range(rin.n_nodes)]
    for r in range(rin.n_rules):
        for n in rn[r]:
            per_node[n].append(r)
    raw = O.jobset(rin)
    raw.rule_key = None
    L = O.lib()
    shadowed = sum(L.or_rule_on_node(raw, mode, r, n) for r in range(rin.n_rules) for n in range(rin.n_nodes)) \
        - sum(len(p) for p in per_node)
    assert shadowed > 0
    for n in range(rin.n_nodes):
        if mode == _lib.EXCLUDE_NONE:
            nid = js.node_id(n)
            cmds = sorted(r for j in range(len(js.jobs)) for r in js.cmds(j, nid))
            assert cmds == per_node[n], n
        exp_t, exp_r = O.node_list(eo, et, per_node[n]) if per_node[n] else (np.zeros(0, np.int64),
                                                                            np.zeros(0, np.int32))
        if order == "time":
            o = np.lexsort((exp_r, exp_t))
            exp_t, exp_r = exp_t[o], exp_r[o]
        assert np.array_equal(time[node_off[n]:node_off[n + 1]], exp_t), n
        assert np.array_equal(rule[node_off[n]:node_off[n + 1]], exp_r), n


def test_per_node_config3_scale_properties(eng):
    """Config 3 shape at reduced rule count: invariants of the node CSR."""
    rin = synth.rules_for_nodes(50_000)
    specs = synth.spec_mix(rin.n_rules, seed=5, mix=synth.MIX_LIGHT)
    arr, status = cron.parse_batch(specs)
    sp = eng.upload_c(arr, rin.n_rules)
    t0, t1 = synth.T0_2026, synth.T0_2026 + DAY
    node_off, time, rule = eng.expand_per_node(sp, None, t0, t1, rin, _lib.EXCLUDE_NONE)
    roff, rtimes = eng.expand(sp, None, t0, t1)
    cnt = np.diff(roff)
    rn_off, rn_nodes = eng.rule_nodes(rin, _lib.EXCLUDE_NONE)
    # every (rule, node) pair contributes exactly cnt[rule] events
    assert node_off[-1] == int(np.sum(cnt[np.repeat(np.arange(rin.n_rules), np.diff(rn_off))]))
    assert ((time > t0) & (time <= t1)).all()
    # within each node, rules ascend and times ascend within a rule
    for n in np.random.default_rng(1).choice(rin.n_nodes, 50, replace=False):
        r = rule[node_off[n]:node_off[n + 1]]
        assert (np.diff(r) >= 0).all()


def test_device_resident_rules_same_result(eng):
    """cg_rules_upload + cg_expand_per_node_rules_device == the host-array path."""
    rin = synth.multi_rule_jobs(200, seed=31)
    specs = synth.spec_mix(rin.n_rules, seed=8, mix=synth.MIX_LIGHT)
    arr, status = cron.parse_batch(specs)
    sp = eng.upload_c(arr, rin.n_rules)
    t0, t1 = synth.T0_2026, synth.T0_2026 + DAY
    for mode in (_lib.EXCLUDE_NONE, _lib.EXCLUDE_RULE, _lib.EXCLUDE_CUMULATIVE):
        node_off, time, rule = eng.expand_per_node(sp, None, t0, t1, rin, mode)
        drules = eng.upload_rules(rin)
        for _ in range(2):  # reusable without re-upload
            En, nnz = eng.expand_per_node_rules_device(sp, None, t0, t1, drules, mode)
            o2, t2, r2 = eng.node_result(rin.n_nodes, En)
            assert np.array_equal(o2, node_off) and np.array_equal(t2, time)
            assert np.array_equal(r2, rule)
        drules.free()


def test_transpose_cache_keyed_by_rule_set_and_mode(eng):
    """The rule->node join + transpose is reused across calls on the same
    uploaded rule set and mode (time windows); switching rule set or mode, or
    interleaving the host-array path, must never reuse a stale transpose."""
    ra = synth.multi_rule_jobs(150, seed=41)
    rb = synth.multi_rule_jobs(150, seed=42)
    t0 = synth.T0_2026
    fresh = {}
    sps = {}
    for name, rin in (("a", ra), ("b", rb)):
        specs = synth.spec_mix(rin.n_rules, seed=9, mix=synth.MIX_LIGHT)
        arr, _ = cron.parse_batch(specs)
        sps[name] = eng.upload_c(arr, rin.n_rules)
        for mode in (_lib.EXCLUDE_NONE, _lib.EXCLUDE_CUMULATIVE):
            for w in range(2):
                a = t0 + w * 3600
                fresh[name, mode, w] = eng.expand_per_node(sps[name], None, a, a + 3600, rin, mode)
    da, db = eng.upload_rules(ra), eng.upload_rules(rb)
    order = [("a", 0, 0), ("a", 0, 1), ("b", 0, 0), ("a", 2, 1), ("a", 2, 0), ("a", 0, 1),
             ("b", 2, 1), ("b", 2, 0)]
    for name, mode, w in order:
        rin, d = (ra, da) if name == "a" else (rb, db)
        a = t0 + w * 3600
        En, _ = eng.expand_per_node_rules_device(sps[name], None, a, a + 3600, d, mode)
        got = eng.node_result(rin.n_nodes, En)
        exp = fresh[name, mode, w]
        assert all(np.array_equal(x, y) for x, y in zip(got, exp)), (name, mode, w)
        if w == 1:  # the host-array path in between re-uploads its own rule set
            eng.expand_per_node(sps[name], None, a, a + 3600, rin, mode)


def _ordered_per_node(eng, writer, scheds, zone, t0, t1, rin):
    """The per-node result in (time, rule) order: "pass" = rule-major lists,
    then cg_node_result_order_by_time; "direct" = cg_set_node_order(TIME)
    (the pass inside the per-node call).  Returns the rule-major node offsets
    and the ordered CSR."""
    if writer == "direct":
        eng.set_node_order(_lib.NODE_ORDER_TIME)
        try:
            node_off, time, rule = eng.expand_per_node(scheds, zone, t0, t1, rin, _lib.EXCLUDE_NONE)
        finally:
            eng.set_node_order(_lib.NODE_ORDER_RULE)
        assert eng.node_order_by_time() == 0.0  # already ordered: nothing to do
        return node_off, node_off, time, rule
    node_off, time, rule = eng.expand_per_node(scheds, zone, t0, t1, rin, _lib.EXCLUDE_NONE)
    ms = eng.node_order_by_time()
    assert ms >= 0
    off2, time2, rule2 = eng.node_result(rin.n_nodes, len(time))
    return node_off, off2, time2, rule2


@pytest.mark.parametrize("writer", ["pass", "direct"])
@pytest.mark.parametrize("zone,t0,secs", [("UTC", synth.T0_2026 + 64 * DAY, 3600), ("UTC", synth.T0_2026, 25 * 3600),
                                          ("America/New_York", 1772953200 - 12 * 3600, 24 * 3600),
                                          ("America/New_York", 1772953200 - 1800, 4096),
                                          ("UTC", synth.T0_2026 + 7 * 3600 + 13, 61),
                                          ("UTC", synth.T0_2026 + 5 * 3600 + 59, 1)])
def test_per_node_time_ordered_vs_oracle(eng, writer, zone, t0, secs):
    """Every node's list in (time, rule) order -- the byTime order of Cron.run
    (cron.go:64-79,220) with equal times in rule order -- against the
    oracle's per-node lists.  "pass": cg_node_result_order_by_time over the
    rule-major lists (windows <= 4096 s by the tile sort + merge, longer ones
    by 3 radix passes); "direct": cg_set_node_order(TIME), the same passes
    inside the per-node call (1 h, 4096 s across the NY spring-forward, 61 s,
    1 s, 24-25 h).  Node offsets equal the rule-major ones."""
    hours = secs / 3600
    rin = synth.multi_rule_jobs(300, seed=23)
    specs = synth.spec_mix(rin.n_rules, seed=6, mix=synth.MIX_CONFIG2)
    scheds = [cron.Parse(s) for s in specs]
    t1 = t0 + secs
    node_off, off2, time2, rule2 = _ordered_per_node(eng, writer, scheds, product_zone(zone), t0, t1, rin)
    time = time2
    assert np.array_equal(off2, node_off)
    arr = O.sched_array(oracle_parse_all(specs))
    eo, et = O.expand_batch(arr, t0, t1, oracle_zone(zone))
    rn = oracle_rule_nodes(rin, _lib.EXCLUDE_NONE)
    per_node = [[] for _ in range(rin.n_nodes)]
    for r in range(rin.n_rules):
        for n in rn[r]:
            per_node[n].append(r)
    checked = 0
    for n in range(rin.n_nodes):
        exp_t, exp_r = O.node_list(eo, et, per_node[n]) if per_node[n] else (np.zeros(0, np.int64),
                                                                            np.zeros(0, np.int32))
        order = np.lexsort((exp_r, exp_t))
        a, b = node_off[n], node_off[n + 1]
        assert np.array_equal(time2[a:b], exp_t[order]), n
        assert np.array_equal(rule2[a:b], exp_r[order]), n
        checked += b - a
    assert checked == len(time) > (1000 if hours >= 1 else (100 if secs > 1 else 10))


PROGRESSION_MIX = ["* * * * * *", "*/13 * * * * *", "@every 7s", "@every 1h", "@every 90m", "0 0 * * * *",
                   "0 30 9 * * *", "0 0 0 * * *", "0 */20 * * * *", "0 7,30,45 * * * *", "0 0 12 * * 1",
                   "0 0 0 30 2 *", "15 * * * * *"]


def progression_rules(R, n_nodes):
    """Rules on two nodes each (no groups): rule i on nodes i % N and (7i + 1) % N."""
    from cronsun_amd.engine import RulesIn
    nids = np.stack([np.arange(R) % n_nodes, (7 * np.arange(R) + 1) % n_nodes], 1)
    nids = np.sort(nids, 1)
    same = nids[:, 0] == nids[:, 1]  # one node: listed once
    nid_off = np.zeros(R + 1, np.int64)
    nid_off[1:] = np.cumsum(np.where(same, 1, 2))
    keep = np.ones((R, 2), bool)
    keep[:, 1] = ~same
    z = np.zeros(R + 1, np.int64)
    return RulesIn(n_nodes, 0, R, R, group_off=np.zeros(1, np.int64), group_nodes=np.zeros(0, np.int32),
                   group_exists=np.zeros(0, np.uint8), rule_job=np.arange(R, dtype=np.int32), nid_off=nid_off,
                   nids=nids[keep].astype(np.int32), gid_off=z,
                   gids=np.zeros(0, np.int32), ex_off=z, ex=np.zeros(0, np.int32),
                   job_pause=np.zeros(R, np.uint8))


@pytest.mark.parametrize("writer", ["pass", "direct"])
@pytest.mark.parametrize("R,N,secs,star_every", [(1200, 3, 3600, 13), (2600, 2, 4096, 2), (64, 1, 61, 3),
                                                 (12000, 1, 120, 1), (40, 1, 4096, 10**9), (200, 1, 3600, 2),
                                                 (1200, 1, 1800, 1), (2600, 2, 2048, 2)])
def test_per_node_time_ordered_big_nodes(eng, writer, R, N, secs, star_every):
    """The one-pass time order on nodes far larger than one LDS chunk:
    every-second rules put > 4096 events into one 64-s slab (the slab is
    histogrammed, then stored chunk by chunk at its digits' running bases),
    and at 2600 rules on 2 nodes over 4096 s each node holds > 5 M events,
    more than 1024 tiles (portion lists in groups); 61 s: one tile per node.
    12000 every-second rules on one node: every second holds more events than
    a merge chunk (k_ot_big sorts the slab chunk by chunk).  40 sparse rules
    on one node over 4096 s: ~7 k events in two tiles, merge runs of dozens of
    slabs (sorted in two 8-bit passes).  200 rules on one node, every other one
    every second, over 1 h: ~6.5 k events per slab, each merged by k_ot_mid's
    8192-event chunk.  Windows <= 2048 s (32-s slabs): 1200 every-second
    rules on one node over 30 min (38 k events per slab -> k_ot_big), 2600
    rules on 2 nodes over 2048 s (> 1024 tiles per node).
    Against the oracle's lists sorted by (time, rule)."""
    specs = [PROGRESSION_MIX[0] if i % star_every == 0 else PROGRESSION_MIX[1 + i % (len(PROGRESSION_MIX) - 1)]
             for i in range(R)]
    rin = progression_rules(R, N)
    scheds = [cron.Parse(s) for s in specs]
    t0 = synth.T0_2026 + 9 * DAY + 777
    t1 = t0 + secs
    node_off, off2, time2, rule2 = _ordered_per_node(eng, writer, scheds, product_zone("UTC"), t0, t1, rin)
    assert np.array_equal(off2, node_off)
    arr = O.sched_array(oracle_parse_all(specs))
    eo, et = O.expand_batch(arr, t0, t1, oracle_zone("UTC"))
    rn = oracle_rule_nodes(rin, _lib.EXCLUDE_NONE)
    per_node = [[] for _ in range(N)]
    for r in range(R):
        for n in rn[r]:
            per_node[n].append(r)
    for n in range(N):
        exp_t, exp_r = O.node_list(eo, et, per_node[n])
        order = np.lexsort((exp_r, exp_t))
        a, b = node_off[n], node_off[n + 1]
        assert b - a == len(exp_t), n
        assert np.array_equal(time2[a:b], exp_t[order]), n
        assert np.array_equal(rule2[a:b], exp_r[order]), n
    if R == 2600 and secs == 4096:
        assert (np.diff(node_off) > 1024 * 4096).all()
    if R == 200:  # every slab between a merge chunk and a k_ot_mid chunk
        per_slab = node_off[1] / (secs / 64)
        assert 4096 < per_slab < 8192 and node_off[1] < 256 * 4096
    if R == 40:  # two tiles, runs of more than 4 slabs
        assert 4096 < node_off[1] < 2 * 4096 and node_off[1] < 64 * 4096 // 8


@pytest.mark.parametrize("writer", ["pass", "direct"])
@pytest.mark.parametrize("case", ["mid", "dense", "mid2"])
@pytest.mark.parametrize("secs", [3600, 1800])
def test_per_node_time_ordered_slab_classes(eng, writer, case, secs):
    """Each path of the merge by slab size, on one node over 1 h (64-s slabs)
    and over 30 min (windows <= 2048 s: 32-s slabs, ot_slab_bits), against
    the oracle's (time, rule) lists; k = 64 / slab width rules per unit:
    mid    a sparse node (<= 2048 events per 64 s on average, 4-wave merge)
           with one heavy slab: 100 k rules every second of minute 5 put
           > 4096 events into one slab -> k_ot_mid (8-wave, 8192 events);
    dense  100 k every-second rules among 200 k: > 2048 events per 64 s on
           average -> the 8-wave merge (persistent grid, own stream);
    mid2   200 k every-second rules among 400 k: ~13 k per slab -> k_ot_mid's
           16-wave form (16384 events)."""
    w = 64 if secs > 2048 else 32
    k = 64 // w
    mix = PROGRESSION_MIX[1:]
    if case == "mid":
        specs = ["* 5 * * * *" if i % 2 == 0 else mix[i % len(mix)] for i in range(200 * k)]
    else:
        R = (200 if case == "dense" else 400) * k
        specs = [PROGRESSION_MIX[0] if i % 2 == 0 else mix[i % len(mix)] for i in range(R)]
    rin = progression_rules(len(specs), 1)
    scheds = [cron.Parse(x) for x in specs]
    t0 = synth.T0_2026 + 11 * DAY + 297  # minute 5 of the hour at offsets 2..61
    t1 = t0 + secs
    node_off, off2, time2, rule2 = _ordered_per_node(eng, writer, scheds, product_zone("UTC"), t0, t1, rin)
    assert np.array_equal(off2, node_off)
    arr = O.sched_array(oracle_parse_all(specs))
    eo, et = O.expand_batch(arr, t0, t1, oracle_zone("UTC"))
    exp_t, exp_r = O.node_list(eo, et, list(range(len(specs))))
    order = np.lexsort((exp_r, exp_t))
    assert node_off[1] == len(exp_t)
    assert np.array_equal(time2, exp_t[order])
    assert np.array_equal(rule2, exp_r[order])
    per_slab = np.bincount((exp_t - t0 - 1) // w)
    avg = len(exp_t) / np.ceil(secs / 64)  # the dense split's events per 64 s
    if case == "mid":
        assert avg <= 2048 and 4096 < per_slab.max() <= 8192
    elif case == "dense":
        assert avg > 2048 and per_slab.max() <= 8192
    else:
        assert 8192 < per_slab.max() <= 16384


@pytest.mark.parametrize("zone,t0", [("UTC", synth.T0_2026 + 64 * DAY + 1234),
                                     ("America/New_York", 1772953200 - 36 * 3600)])
def test_per_node_progressions_vs_oracle(eng, zone, t0):
    """The per-node writer's computed fires (k_rule_info / k_seg_records
    progression records: t0 + x + p * stride) against the oracle: every-second,
    @every, hourly, daily (a 23/25-h step across the NY DST change breaks the
    progression), weekly, never-firing and non-progression rules, over 3 days
    and 3 rule bands, with every-second rules early in a node's band so the
    positions of later daily rules overflow the record's 32-bit x (those fall
    back to gathers)."""
    R, N = 2600, 6
    specs = [PROGRESSION_MIX[1 + i % (len(PROGRESSION_MIX) - 1)] for i in range(R)]
    for i in (0, 1, 1030, 2100):  # a few every-second rules (259 200 fires each), early in bands
        specs[i] = PROGRESSION_MIX[0]
    rin = progression_rules(R, N)
    scheds = [cron.Parse(s) for s in specs]
    t1 = t0 + 3 * DAY
    node_off, time, rule = eng.expand_per_node(scheds, product_zone(zone), t0, t1, rin, _lib.EXCLUDE_NONE)
    arr = O.sched_array(oracle_parse_all(specs))
    eo, et = O.expand_batch(arr, t0, t1, oracle_zone(zone))
    rn = oracle_rule_nodes(rin, _lib.EXCLUDE_NONE)
    per_node = [[] for _ in range(N)]
    for r in range(R):
        for n in rn[r]:
            per_node[n].append(r)
    for n in range(N):
        exp_t, exp_r = O.node_list(eo, et, per_node[n])
        assert np.array_equal(time[node_off[n]:node_off[n + 1]], exp_t), n
        assert np.array_equal(rule[node_off[n]:node_off[n + 1]], exp_r), n


@pytest.mark.parametrize("order", ["rule", "time"])
@pytest.mark.parametrize("zone", ["UTC", "America/New_York"])
def test_per_node_async_windows(zone, order):
    """cg_expand_per_node_rules_device_async / cg_expand_per_node_wait: a node
    scheduler's consecutive windows (node/node.go:121-158 + cron.go:210-275),
    pipelined.  The last window's per-node CSR equals the synchronous result of
    that window and the oracle; the all-window total equals the sum of the
    windows' synchronous totals; accessors refuse while windows are pending; a
    window beyond the capacity reports CG_ECAPACITY at the wait; a synchronous
    call in between discards pending windows.  order "time"
    (cg_set_node_order): every window's tile sort + merge enqueued behind its
    writer, the last window against the oracle's lists in (time, rule) order;
    windows over 4096 s are refused at the call."""
    from cronsun_amd.engine import Engine
    from cronsun_amd._lib import check, lib
    e2 = Engine(0)
    timed = order == "time"
    if timed:
        e2.set_node_order(_lib.NODE_ORDER_TIME)
    rin = synth.multi_rule_jobs(2000, seed=31)
    specs = synth.spec_mix(rin.n_rules, seed=9, mix=synth.MIX_CONFIG2)
    arr, status = cron.parse_batch(specs)
    assert (status == 0).all()
    sp = e2.upload_c(arr, rin.n_rules)
    dr = e2.upload_rules(rin)
    z = product_zone(zone)
    t0 = 1772953200 - 5 * 3600 if zone != "UTC" else synth.T0_2026 + 3 * 3600 + 17
    e2.expand_per_node_rules_device(sp, z, t0, t0 + 3 * 3600, dr, _lib.EXCLUDE_NONE)  # sizes the outputs
    wins = [(t0 + 1800 * i, t0 + 1800 * i + 3600) for i in range(8)]
    for a, b in wins:
        e2.expand_per_node_async(sp, z, a, b, dr, _lib.EXCLUDE_NONE)
    with pytest.raises(_lib.CgError) as err:
        e2.node_copy_range(0, 1)
    assert err.value.code == _lib.CG_EINVAL
    En, tot = e2.expand_per_node_wait(with_total=True)
    off = np.empty(rin.n_nodes + 1, np.int64)
    check(lib().cg_node_result_copy(e2._h, off.ctypes.data, None, None, 0))
    got_t, got_r = e2.node_copy_range(0, En)
    sync_tot = 0
    for a, b in wins:
        Ew, _ = e2.expand_per_node_rules_device(sp, z, a, b, dr, _lib.EXCLUDE_NONE)
        sync_tot += Ew
    assert tot == sync_tot
    assert En == Ew
    off_s = np.empty_like(off)
    check(lib().cg_node_result_copy(e2._h, off_s.ctypes.data, None, None, 0))
    st_t, st_r = e2.node_copy_range(0, Ew)
    assert np.array_equal(off, off_s) and np.array_equal(got_t, st_t) and np.array_equal(got_r, st_r)
    # the oracle, every node, last window
    a, b = wins[-1]
    eo, et = O.expand_batch(O.sched_array(oracle_parse_all(specs)), a, b, oracle_zone(zone))
    rn = oracle_rule_nodes(rin, _lib.EXCLUDE_NONE)
    per_node = [[] for _ in range(rin.n_nodes)]
    for r in range(rin.n_rules):
        for n in rn[r]:
            per_node[n].append(r)
    for n in range(rin.n_nodes):
        if not per_node[n]:
            assert off[n + 1] == off[n]
            continue
        exp_t, exp_r = O.node_list(eo, et, per_node[n])
        if timed:
            o = np.lexsort((exp_r, exp_t))
            exp_t, exp_r = exp_t[o], exp_r[o]
        assert np.array_equal(got_t[off[n]:off[n + 1]], exp_t), n
        assert np.array_equal(got_r[off[n]:off[n + 1]], exp_r), n
    if timed:
        with pytest.raises(_lib.CgError) as err:
            e2.expand_per_node_async(sp, z, t0, t0 + 2 * DAY, dr, _lib.EXCLUDE_NONE)
        assert err.value.code == _lib.CG_EINVAL
        dr.free()
        sp.free()
        e2.close()
        # a 4096-s window past the output capacity that a 300-s window sized:
        # the writer and the time-order pass write nothing, CG_ECAPACITY at
        # the wait, and the engine still gives the right result afterwards
        e3 = Engine(0)
        e3.set_node_order(_lib.NODE_ORDER_TIME)
        sp3, dr3 = e3.upload_c(arr, rin.n_rules), e3.upload_rules(rin)
        Es, _ = e3.expand_per_node_rules_device(sp3, z, t0, t0 + 300, dr3, _lib.EXCLUDE_NONE)
        ref = e3.node_copy_range(0, Es)
        e3.expand_per_node_async(sp3, z, t0, t0 + 4096, dr3, _lib.EXCLUDE_NONE)
        with pytest.raises(_lib.CgError) as err:
            e3.expand_per_node_wait()
        assert err.value.code == _lib.CG_ECAPACITY
        e3.expand_per_node_async(sp3, z, t0, t0 + 300, dr3, _lib.EXCLUDE_NONE)
        assert e3.expand_per_node_wait() == Es
        got = e3.node_copy_range(0, Es)
        assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
        dr3.free()
        sp3.free()
        e3.close()
        return
    # a window far beyond the capacity: CG_ECAPACITY at the wait
    e2.expand_per_node_async(sp, z, t0, t0 + 2 * DAY, dr, _lib.EXCLUDE_NONE)
    with pytest.raises(_lib.CgError) as err:
        e2.expand_per_node_wait()
    assert err.value.code == _lib.CG_ECAPACITY
    # a synchronous call discards pending windows (and their errors)
    e2.expand_per_node_async(sp, z, t0, t0 + 2 * DAY, dr, _lib.EXCLUDE_NONE)
    Es, _ = e2.expand_per_node_rules_device(sp, z, a, b, dr, _lib.EXCLUDE_NONE)
    e2.expand_per_node_async(sp, z, a, b, dr, _lib.EXCLUDE_NONE)
    assert e2.expand_per_node_wait() == Es
    dr.free()
    sp.free()
    e2.close()


def test_per_node_bands_past_2_30_fires():
    """A window whose 1024-rule bands hold more than 2^30 fires (1024
    every-second rules over 13 days: 1.15 G fires): the per-node path narrows
    its bands instead of refusing, and sampled nodes' lists are bit-exact
    against the oracle (job.go:591-614 composed with spec.go:55-145 over the
    whole window)."""
    from cronsun_amd.engine import Engine
    e2 = Engine(0)
    R, N = 1100, 48
    specs = ["* * * * * *"] * 1024 + [PROGRESSION_MIX[1 + i % (len(PROGRESSION_MIX) - 1)] for i in range(R - 1024)]
    rin = progression_rules(R, N)
    arr, status = cron.parse_batch(specs)
    assert (status == 0).all()
    sp = e2.upload_c(arr, R)
    dr = e2.upload_rules(rin)
    t0 = synth.T0_2026 + 1234
    t1 = t0 + 13 * DAY
    En, nnz = e2.expand_per_node_rules_device(sp, cron.UTC(), t0, t1, dr, _lib.EXCLUDE_NONE)
    assert En > 2 * (1 << 30)
    from cronsun_amd._lib import check, lib
    off = np.empty(N + 1, np.int64)
    check(lib().cg_node_result_copy(e2._h, off.ctypes.data, None, None, 0))
    rn = oracle_rule_nodes(rin, _lib.EXCLUDE_NONE)
    per_node = [[] for _ in range(N)]
    for r in range(R):
        for n in rn[r]:
            per_node[n].append(r)
    for n in (5, 31):
        rules = per_node[n]
        arr_o = O.sched_array(oracle_parse_all([specs[r] for r in rules]))
        eo, et = O.expand_batch(arr_o, t0, t1, oracle_zone("UTC"), threads=16)
        exp_t, exp_r = O.node_list(eo, et, list(range(len(rules))))
        got_t, got_r = e2.node_copy_range(off[n], off[n + 1] - off[n])
        assert np.array_equal(got_t, exp_t), n
        assert np.array_equal(got_r, np.array(rules, np.int32)[exp_r]), n
    dr.free()
    sp.free()
    e2.close()


@pytest.mark.parametrize("writer,R", [("pass", (1 << 20) + 50_000), ("direct", (1 << 20) + 50_000),
                                      ("direct", (1 << 24) + 50_000)])
def test_per_node_time_ordered_over_2_20_rules(writer, R):
    """More than 2^20 rules: (offset, rule) no longer fits one 32-bit word.
    "direct" below 2^24 rules: the writer's packed words hold rule & 0xFFFFF,
    the tiles are cut where rule >> 20 changes (at band boundaries) and carry
    those bits, and the merges rebuild the rule from the tile (keys rel << 24
    | rule).  "direct" past 2^24: 16-bit offsets + rules, the tile sort and
    merges keep an LDS rule array; "pass": the separate pass over the int64
    lists (unpacked).  134 every-second rules per 2^20 (all on nodes 0 and 1:
    ~8.6 k events per 64-s slab there, the dense merge and k_ot_mid's 16-wave
    form, whose 16384-event chunks need 14 index bits) and every-10-s rules
    every 1000 rules among never-firing ones, 10 minutes; four nodes' lists
    (each across every block of 2^20 rules) against the oracle's, sorted by
    (time, rule)."""
    from cronsun_amd.engine import Engine
    N = 64
    kinds = ["0 0 0 1 1 *", "* * * * * *", "*/10 * * * * *"]
    kind = np.zeros(R, np.int64)
    kind[::8192] = 1
    kind[1::1000] = 2
    karr, status = cron.parse_batch(kinds, threads=1)
    assert not np.any(status)
    a = np.ascontiguousarray(np.ctypeslib.as_array(karr)[kind])  # rule i = kinds[kind[i]]
    arr = (karr._type_ * R).from_buffer(a)
    rin = progression_rules(R, N)
    t0 = synth.T0_2026 + 20 * DAY + 123  # January 25: the yearly rules never fire
    t1 = t0 + 600
    eng = Engine(0)
    try:
        sp = eng.upload_c(arr, R)
        dr = eng.upload_rules(rin)
        if writer == "direct":
            eng.set_node_order(_lib.NODE_ORDER_TIME)
        E, _ = eng.expand_per_node_rules_device(sp, product_zone("UTC"), t0, t1, dr, _lib.EXCLUDE_NONE)
        if writer == "pass":
            eng.node_order_by_time()
        off, time, rule = eng.node_result(N, E)
    finally:
        eng.set_node_order(_lib.NODE_ORDER_RULE)
        eng.close()
    assert E > 100_000
    parsed = [O.parse(k)[0] for k in kinds]
    r_all = np.arange(R)
    for n in (0, 1, 37, 63):
        rules_n = r_all[(r_all % N == n) | ((7 * r_all + 1) % N == n)]
        oarr = O.sched_array([parsed[k] for k in kind[rules_n].tolist()])
        eo, et = O.expand_batch(oarr, t0, t1, oracle_zone("UTC"))
        exp_t, exp_p = O.node_list(eo, et, list(range(len(rules_n))))
        exp_r = rules_n[exp_p]
        order = np.lexsort((exp_r, exp_t))
        a, b = int(off[n]), int(off[n + 1])
        assert b - a == len(exp_t), n
        assert np.array_equal(time[a:b], exp_t[order]), n
        assert np.array_equal(rule[a:b], exp_r[order]), n



def test_per_node_time_ordered_over_2_20_rules_big_slabs():
    """Packed words past 2^20 rules through k_ot_big: ~610 every-second rules
    spread over 1.1 M rules (every block of 2^20 holds some), all on both of
    2 nodes, over a 1-h window: each node holds ~2.2 M events in more than
    kOtMaxTiles tiles (every slab to k_ot_big) and 64-s slabs of ~39 k events;
    the tiles are cut where rule >> 20 changes and k_ot_big rebuilds the rule
    from each portion's tile.  Both nodes' whole lists against the oracle's,
    sorted by (time, rule)."""
    from cronsun_amd.engine import Engine
    R, N = (1 << 20) + 50_000, 2
    kinds = ["0 0 0 1 1 *", "* * * * * *"]
    kind = np.zeros(R, np.int64)
    kind[7::1800] = 1
    karr, status = cron.parse_batch(kinds, threads=1)
    assert not np.any(status)
    a = np.ascontiguousarray(np.ctypeslib.as_array(karr)[kind])
    arr = (karr._type_ * R).from_buffer(a)
    rin = progression_rules(R, N)
    t0 = synth.T0_2026 + 20 * DAY + 123
    t1 = t0 + 3600
    eng = Engine(0)
    try:
        sp = eng.upload_c(arr, R)
        dr = eng.upload_rules(rin)
        eng.set_node_order(_lib.NODE_ORDER_TIME)
        E, _ = eng.expand_per_node_rules_device(sp, product_zone("UTC"), t0, t1, dr, _lib.EXCLUDE_NONE)
        off, time, rule = eng.node_result(N, E)
    finally:
        eng.set_node_order(_lib.NODE_ORDER_RULE)
        eng.close()
    fire = np.nonzero(kind == 1)[0]
    assert (fire >> 20).max() == 1 and (fire >> 20).min() == 0  # both blocks of 2^20 rules
    exp_t = np.tile(np.arange(t0 + 1, t1 + 1, dtype=np.int64)[:, None], (1, len(fire))).ravel()
    exp_r = np.tile(fire.astype(np.int32), t1 - t0)  # (time, rule) order: every second, rules ascending
    for n in range(N):
        a_, b_ = int(off[n]), int(off[n + 1])
        assert b_ - a_ == len(exp_t) > 256 * 4096, n
        assert np.array_equal(time[a_:b_], exp_t), n
        assert np.array_equal(rule[a_:b_], exp_r), n


@pytest.mark.parametrize("seed,window", [(1, 600), (2, 1800), (3, 3600)])
def test_time_order_packed_high_bits_equals_unpacked_pass(seed, window):
    """Differential check of the packed time order past 2^20 rules (tiles cut
    where rule >> 20 changes, the merges rebuild the rule from the tile) against
    the independent unpacked path (rule-major int64 lists, then
    cg_node_result_order_by_time: 16-bit offsets + LDS rule arrays), on every
    node's whole list: a random count of rules between 2^20 and 2^21 (the
    config-2 mix, tiled), 37 nodes, 10-min / 30-min / 1-h windows (16-, 32-
    and 64-s slabs)."""
    from cronsun_amd.engine import Engine
    rng = np.random.default_rng(seed)
    R, N = (1 << 20) + int(rng.integers(1, 1 << 20)), 37
    base = synth.spec_mix(50_000, seed=100 + seed, mix=synth.MIX_CONFIG2)
    barr, status = cron.parse_batch(base, threads=16)
    assert not np.any(status)
    pick = rng.integers(0, len(base), R)  # rule r = base[pick[r]]
    a = np.ascontiguousarray(np.ctypeslib.as_array(barr)[pick])
    arr = (barr._type_ * R).from_buffer(a)
    rin = progression_rules(R, N)
    t0 = synth.T0_2026 + int(rng.integers(0, 300)) * DAY + int(rng.integers(0, 86400))
    eng = Engine(0)
    try:
        sp = eng.upload_c(arr, R)
        dr = eng.upload_rules(rin)
        eng.set_node_order(_lib.NODE_ORDER_TIME)
        E1, _ = eng.expand_per_node_rules_device(sp, product_zone("UTC"), t0, t0 + window, dr, _lib.EXCLUDE_NONE)
        got = eng.node_result(N, E1)
        eng.set_node_order(_lib.NODE_ORDER_RULE)
        E2, _ = eng.expand_per_node_rules_device(sp, product_zone("UTC"), t0, t0 + window, dr, _lib.EXCLUDE_NONE)
        eng.node_order_by_time()
        ref = eng.node_result(N, E2)
    finally:
        eng.set_node_order(_lib.NODE_ORDER_RULE)
        eng.close()
    assert E1 == E2 > 1_000_000
    for x, y in zip(got, ref):
        assert np.array_equal(x, y)
    # and two nodes against the oracle's lists sorted by (time, rule)
    off, time, rule = got
    parsed = [O.parse(sp_)[0] for sp_ in base]
    r_all = np.arange(R)
    for n in (0, 19):
        rules_n = r_all[(r_all % N == n) | ((7 * r_all + 1) % N == n)]
        oarr = O.sched_array([parsed[i] for i in pick[rules_n].tolist()])
        eo, et = O.expand_batch(oarr, t0, t0 + window, oracle_zone("UTC"), threads=16)
        exp_t, exp_p = O.node_list(eo, et, list(range(len(rules_n))))
        exp_r = rules_n[exp_p]
        order = np.lexsort((exp_r, exp_t))
        a_, b_ = int(off[n]), int(off[n + 1])
        assert np.array_equal(time[a_:b_], exp_t[order]), n
        assert np.array_equal(rule[a_:b_], exp_r[order]), n
