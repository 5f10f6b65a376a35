"""cronsun's Job/JobRule/Group resolution on the host (C++ cg_jobset behind
cronsun_amd.model) vs the oracle's restatement of job.go:274-288, 591-630,
group.go:111-119 and web/job.go:222-257.  The reference has no tests for this
code, so parity here rests on the oracle and on the hand-derived
fixtures of tests/golden/rule_nodes_cases.py (tests/test_rule_nodes_fixtures.py)."""
import numpy as np
import pytest

import oracle_lib as O
from cronsun_amd import _lib
from cronsun_amd.model import ErrNilRule, Group, Job, JobRule, JobSet


def _oracle_js(rin, keyed=True):
    """The oracle's view of rin; keyed=False drops the Cmd keys (every rule its
    own key), so a test can apply Job.Cmds' map by hand on top."""
    js = O.jobset(rin)
    if not keyed:
        js.rule_key = None
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
    assert rin.rule_key is not None
    ojs, ojs_raw = _oracle_js(rin), _oracle_js(rin, keyed=False)
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
                if n >= 0 and L.or_rule_on_node(ojs_raw, 0, r, n):
                    exp[job.ID + js.rules[r].ID] = r
            assert js.cmds(j, nid) == sorted(exp.values()), (job.ID, nid)
            # the oracle's per-node filter (what the GPU per-node lists are
            # checked against) keeps exactly Job.Cmds' rules
            assert [r for r in rules if n >= 0 and L.or_rule_on_node(ojs, 0, r, n)] == js.cmds(j, nid)
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


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_keyed_oracle_is_cmds_map_in_every_mode(mode):
    """or_rule_on_node with keys = the mode's own inclusion + Job.Cmds' map
    (last scheduled rule per Job.ID+Rule.ID) applied on top."""
    jobs, groups, nodes = random_world(20 + mode, n_jobs=80)
    js = JobSet(jobs, groups)
    rin = js.rules_in()
    ojs, raw = _oracle_js(rin), _oracle_js(rin, keyed=False)
    L = O.lib()
    dropped = 0
    for n in range(rin.n_nodes):
        exp = {}
        for r in range(rin.n_rules):
            if L.or_rule_on_node(raw, mode, r, n):
                exp[(int(rin.rule_job[r]), js.rules[r].ID)] = r
        got = [r for r in range(rin.n_rules) if L.or_rule_on_node(ojs, mode, r, n)]
        assert got == sorted(exp.values()), (mode, n)
        dropped += sum(L.or_rule_on_node(raw, mode, r, n) for r in range(rin.n_rules)) - len(got)
    assert dropped > 0  # the world repeats keys


def test_ingested_duplicate_and_blank_rule_ids():
    """etcd values through the ingest path: Rule.IDs are never trimmed on the
    node path (only Job.Check does, job.go:524-529), so "" repeats "" but not
    " "; cross-job GetID collisions ("j"+"1x" vs "j1"+"x") are kept apart."""
    import json
    from cronsun_amd.ingest import EtcdJobSet
    jobs = [
        {"id": "j", "name": "a", "cmd": "true", "rules": [
            {"id": "", "timer": "@daily", "nids": ["n1", "n2"]},
            {"id": " ", "timer": "@hourly", "nids": ["n1"]},
            {"id": "", "timer": "@weekly", "nids": ["n2", "n3"]},
            {"id": "1x", "timer": "0 * * * * *", "gids": ["g"]}]},
        {"id": "j1", "name": "b", "cmd": "true", "rules": [
            {"id": "x", "timer": "@daily", "nids": ["n1"]},
            {"id": "x", "timer": "@monthly", "gids": ["g"], "exclude_nids": ["n1"]}]},
    ]
    groups = [{"id": "g", "name": "g", "nids": ["n1", "n3"]}]
    js = EtcdJobSet([json.dumps(j) for j in jobs], [json.dumps(g) for g in groups], threads=2)
    rin = js.rules_in()
    assert [js.rule_id(r) for r in range(rin.n_rules)] == [b"", b" ", b"", b"1x", b"x", b"x"]
    ojs = _oracle_js(rin)
    L = O.lib()
    want = {"n1": [[0, 1, 3], [5]], "n2": [[2], []], "n3": [[2, 3], [5]]}
    for nid, per_job in want.items():
        n = js.node_index(nid)
        for j in range(2):
            assert js.cmds(j, nid) == per_job[j], (nid, j)
            rules = [r for r in range(rin.n_rules) if rin.rule_job[r] == j]
            assert [r for r in rules if L.or_rule_on_node(ojs, 0, r, n)] == per_job[j], (nid, j)
    # RULE mode: rule 5 excludes n1, so rule 4 keeps its Cmd there
    n1 = js.node_index("n1")
    assert [r for r in (4, 5) if L.or_rule_on_node(ojs, 1, r, n1)] == [4]


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
