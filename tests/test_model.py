"""cronsun's Job/JobRule/Group resolution on the host (C++ cg_jobset behind
cronsun_amd.model) vs the oracle's restatement of job.go:274-288, 591-630,
group.go:111-119 and web/job.go:222-257.  The reference has no tests for this
code, so parity here is pinned by the oracle only."""
import numpy as np
import pytest

import oracle_lib as O
from cronsun_amd import _lib
from cronsun_amd.model import ErrNilRule, Group, Job, JobRule, JobSet


def _oracle_js(rin):
    js = O.OrJobset()
    js.n_nodes, js.n_groups, js.n_rules, js.n_jobs = rin.n_nodes, rin.n_groups, rin.n_rules, rin.n_jobs
    for f in rin.FIELDS:
        setattr(js, f, getattr(rin, f).ctypes.data)
    return js


def random_world(seed, n_jobs=60, n_nodes=20, n_groups=6):
    rng = np.random.default_rng(seed)
    nodes = [f"10.0.0.{i}" for i in range(n_nodes)]
    groups = {}
    for g in range(n_groups):
        k = int(rng.integers(0, 6))
        groups[f"g{g}"] = Group(f"g{g}", f"group {g}", list(rng.choice(nodes, k, replace=False)))
    jobs = []
    for j in range(n_jobs):
        rules = []
        for r in range(int(rng.integers(1, 5))):
            rid = f"r{rng.integers(0, 3)}"  # duplicates within a job happen
            gids = [f"g{rng.integers(0, n_groups + 2)}" for _ in range(rng.integers(0, 3))]  # g6/g7 missing
            nids = list(rng.choice(nodes, int(rng.integers(0, 4)), replace=False))
            ex = list(rng.choice(nodes, int(rng.integers(0, 3)), replace=False))
            rules.append(JobRule(rid, "0 * * * * *", gids, nids, ex))
        jobs.append(Job(f"job{j:04x}", Rules=rules, Pause=bool(rng.random() < 0.15)))
    return jobs, groups, nodes


@pytest.mark.parametrize("seed", range(5))
def test_cmds_is_run_on_job_nodes_vs_oracle(seed):
    jobs, groups, nodes = random_world(seed)
    js = JobSet(jobs, groups)
    rin = js.rules_in()
    ojs = _oracle_js(rin)
    L = O.lib()
    rule0 = 0
    for j, job in enumerate(jobs):
        rules = list(range(rule0, rule0 + len(job.Rules)))
        rule0 += len(job.Rules)
        for nid in nodes + ["unknown-node"]:
            n = js.node_index(nid)
            # Job.Cmds: map keyed by Job.ID+Rule.ID, later rules overwrite
            exp = {}
            for r in rules:
                if n >= 0 and L.or_rule_on_node(ojs, 0, r, n):
                    exp[job.ID + js.rules[r].ID] = r
            assert js.cmds(j, nid) == sorted(exp.values()), (job.ID, nid)
            exp_run = bool(n >= 0 and L.or_job_is_run_on(ojs, j, n))
            assert js.is_run_on(j, nid) == exp_run
        cap = 256
        buf = (O.C.c_int32 * cap)()
        k = L.or_job_nodes(ojs, j, buf, cap)
        assert js.job_nodes(j) == [js.node_id(buf[i]) for i in range(k)]


def test_exclude_is_a_noop_in_cmds_but_not_in_web_view():
    # job.go:598-602: `continue` only continues the inner loop over excludes
    g = {"web": Group("web", "web", ["n1", "n2", "n3"])}
    job = Job("j1", Rules=[JobRule("a", "@hourly", GroupIDs=["web"], ExcludeNodeIDs=["n2"])])
    assert set(job.Cmds("n2", g)) == {"j1a"}          # still scheduled on n2
    assert job.IsRunOn("n2", g)
    assert job.GetJobNodes(g) == ["n1", "n3"]          # the web view subtracts it


def test_cumulative_excludes_and_first_seen_order():
    g = {"A": Group("A", "", ["n3", "n1"]), "B": Group("B", "", ["n2", "n4"])}
    job = Job("j", Rules=[JobRule("1", "@daily", GroupIDs=["A"], NodeIDs=["n5"]),
                          JobRule("2", "@daily", GroupIDs=["B"], ExcludeNodeIDs=["n4", "n5"]),
                          JobRule("3", "@daily", NodeIDs=["n4", "n1"])])
    # rule1: n5 n3 n1 ; rule2: (prev + n2 n4) - {n4,n5}; rule3: (prev + n4 n1) - {n4,n5}
    assert job.GetJobNodes(g) == ["n5", "n3", "n1", "n2"]


def test_pause_and_missing_groups():
    g = {"A": Group("A", "", ["n1"])}
    job = Job("j", Pause=True, Rules=[JobRule("1", "@daily", GroupIDs=["A", "missing"])])
    assert job.Cmds("n1", g) == {}          # job.go:593
    assert job.IsRunOn("n1", g)             # IsRunOn ignores Pause
    job.Pause = False
    assert set(job.Cmds("n1", g)) == {"j1"}
    assert not job.IsRunOn("n9", g)


def test_duplicate_rule_ids_last_included_wins():
    g = {}
    job = Job("j", Rules=[JobRule("x", "@daily", NodeIDs=["n1"]), JobRule("x", "@hourly", NodeIDs=["n1"]),
                          JobRule("x", "@weekly", NodeIDs=["n2"])])
    cmds = job.Cmds("n1", g)
    assert list(cmds) == ["jx"] and cmds["jx"][1].Timer == "@hourly"


def test_rule_valid():
    r = JobRule("r", "")
    with pytest.raises(ErrNilRule):
        r.Valid()
    r = JobRule("r", "0 0 * * * *")
    r.Valid()
    assert r.Schedule is not None
    from cronsun_amd.cron import ParseError
    with pytest.raises(ParseError) as e:
        JobRule("r", "bogus spec").Valid()
    assert "invalid JobRule[bogus spec], parse err:" in str(e.value)


def test_rules_in_arrays_consistent():
    jobs, groups, nodes = random_world(9)
    rin = JobSet(jobs, groups).rules_in()
    assert rin.n_rules == sum(len(j.Rules) for j in jobs)
    assert rin.nid_off[-1] == len(rin.nids) or rin.nid_off[-1] == 0
    assert (np.diff(rin.rule_job[:rin.n_rules]) >= 0).all()
