"""Rule -> node resolution against hand-derived fixtures
(tests/golden/rule_nodes_cases.py: worked out from job.go:274-288, 591-614,
group.go:111-119 and web/job.go:222-257 by reading, since the reference has no
tests for this code).  CPU: the oracle in all three exclude modes, and in mode
NONE the Python model's Job.Cmds and the host jobset (cg_jobset_cmds); GPU:
the per-node lists of cg_expand_per_node in all three modes."""
import os
import sys

import numpy as np
import pytest

import oracle_lib as O
from cronsun_amd import _lib, cron
from cronsun_amd.model import Group, Job, JobRule, JobSet

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from rule_nodes_cases import CASES  # noqa: E402

TIMER = "* * * * * *"  # every rule fires every second: each scheduled rule shows in a node's list
MODES = [("none", _lib.EXCLUDE_NONE), ("rule", _lib.EXCLUDE_RULE), ("cumulative", _lib.EXCLUDE_CUMULATIVE)]


def _world(case):
    groups = {g: Group(g, g, list(n)) for g, n in case["groups"].items()}
    jobs, objs = [], []
    for j in case["jobs"]:
        rules = [JobRule(r["id"], TIMER, list(r["gids"]), list(r["nids"]), list(r["ex"])) for r in j["rules"]]
        objs += rules
        jobs.append(Job(j["id"], Rules=rules, Pause=j["pause"]))
    return jobs, groups, objs


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_and_host_vs_fixture(case):
    jobs, groups, objs = _world(case)
    js = JobSet(jobs, groups)
    rin = js.rules_in()
    R = rin.n_rules
    assert R == len(objs)
    ojs = O.jobset(rin)
    L = O.lib()
    for name, mode in MODES:
        for nid, want in case["expected"][name].items():
            n = js.node_index(nid)
            got = [r for r in range(R) if n >= 0 and L.or_rule_on_node(ojs, mode, r, n)]
            assert got == want, (name, nid)
    index = {id(r): i for i, r in enumerate(objs)}
    for nid, want in case["expected"]["none"].items():
        model = sorted(index[id(cmd[1])] for job in jobs for cmd in job.Cmds(nid, groups).values())
        assert model == want, nid
        host = sorted(r for j in range(len(jobs)) for r in js.cmds(j, nid))
        assert host == want, nid


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["rule", "time"])
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_per_node_lists_vs_fixture(case, order):
    from cronsun_amd.engine import Engine
    jobs, groups, objs = _world(case)
    js = JobSet(jobs, groups)
    rin = js.rules_in()
    scheds = [cron.Parse(TIMER) for _ in objs]
    t0 = 1767571200 + 3 * 3600 + 17
    eng = Engine(0)
    try:
        if order == "time":
            eng.set_node_order(_lib.NODE_ORDER_TIME)
        for name, mode in MODES:
            node_off, time, rule = eng.expand_per_node(scheds, None, t0, t0 + 60, rin, mode)
            for nid, want in case["expected"][name].items():
                n = js.node_index(nid)
                a, b = int(node_off[n]), int(node_off[n + 1])
                assert sorted(set(rule[a:b].tolist())) == want, (name, nid)
                assert b - a == 60 * len(want), (name, nid)  # every scheduled rule: its 60 fires
                t, r = time[a:b], rule[a:b]
                if order == "time":
                    assert np.all((np.diff(t) > 0) | ((np.diff(t) == 0) & (np.diff(r) > 0)))
                else:
                    assert np.all((np.diff(r) > 0) | ((np.diff(r) == 0) & (np.diff(t) > 0)))
    finally:
        eng.close()
