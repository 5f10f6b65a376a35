"""BASELINE config 1: 10 000 random six-field specs, UTC,
1 h from 2026-01-05, one group of all 16 nodes.  The golden fixture
(tests/golden/config1.npz, made by tests/golden/gen_config1.py from the
oracle) pins per-rule fire counts and order-sensitive checksums; the CPU test
re-derives them with the oracle, the GPU test with the product (rule-major
and per node)."""
import os
import sys

import numpy as np
import pytest

import oracle_lib as O

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import gen_config1 as G  # noqa: E402

FIX = np.load(os.path.join(HERE, "golden", "config1.npz"))


def test_fixture_inputs_are_the_generator():
    assert list(FIX["specs"]) == G.specs()


def test_oracle_matches_golden():
    scheds = [O.parse(str(s))[0] for s in FIX["specs"]]
    off, times = O.expand_batch(O.sched_array(scheds), int(FIX["t0"]), int(FIX["t1"]), O.Loc("UTC"))
    cnt, s1, s2 = G.checksums(off, times)
    assert np.array_equal(cnt, FIX["count"]) and np.array_equal(s1, FIX["sum"])
    assert np.array_equal(s2, FIX["wsum"])


@pytest.mark.gpu
def test_gpu_matches_golden_rule_major_and_per_node():
    from cronsun_amd import cron
    from cronsun_amd.engine import Engine, RulesIn
    eng = Engine(0)
    arr, status = cron.parse_batch([str(s) for s in FIX["specs"]])
    assert (status == 0).all()
    R, N = len(FIX["specs"]), int(FIX["n_nodes"])
    sp = eng.upload_c(arr, R)
    t0, t1 = int(FIX["t0"]), int(FIX["t1"])
    off, times = eng.expand(sp, None, t0, t1)
    cnt, s1, s2 = G.checksums(off, times)
    assert np.array_equal(cnt, FIX["count"]) and np.array_equal(s1, FIX["sum"])
    assert np.array_equal(s2, FIX["wsum"])
    # one group holding every node; each rule names it
    rin = RulesIn(N, 1, R, R, group_off=np.array([0, N]), group_nodes=np.arange(N),
                  group_exists=np.ones(1), rule_job=np.arange(R), nid_off=np.zeros(R + 1),
                  nids=np.zeros(0), gid_off=np.arange(R + 1), gids=np.zeros(R),
                  ex_off=np.zeros(R + 1), ex=np.zeros(0), job_pause=np.zeros(R))
    node_off, ntime, nrule = eng.expand_per_node(sp, None, t0, t1, rin)
    E = int(off[-1])
    assert np.array_equal(node_off, np.arange(N + 1) * E)
    for n in range(N):
        assert np.array_equal(ntime[n * E:(n + 1) * E], times)
        assert np.array_equal(nrule[n * E:(n + 1) * E], np.repeat(np.arange(R), np.diff(off)))
