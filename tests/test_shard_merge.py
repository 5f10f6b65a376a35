"""shard.merge_rank_runs on host tensors (the numpy path of the time-ordered
gather, CPU): every node's rank slices, each in (time, rule) order with rank
g's global rules below rank g+1's, merge into the node's (time, rule) list --
the byTime order of one Cron over every job (cron.go:64-79,220).  Random runs
with ties across ranks, empty runs and empty nodes; world 1 is a no-op."""
import numpy as np
import pytest
import torch

from cronsun_amd import shard


def _runs(rng, N, W):
    bounds = np.zeros((N, W + 1), np.int64)
    times, rules, pos = [], [], 0
    for n in range(N):
        bounds[n, 0] = pos
        for g in range(W):
            k = int(rng.integers(0, 40)) if rng.random() > 0.2 else 0
            t = np.sort(rng.integers(0, 30, k)) + 1_767_571_200  # few distinct seconds: ties across ranks
            r = np.sort(rng.integers(0, 100, k)) + 100 * g       # rank g's rules below rank g+1's
            o = np.lexsort((r, t))
            times.append(t[o]); rules.append(r[o].astype(np.int32))
            pos += k
            bounds[n, g + 1] = pos
    return bounds, np.concatenate(times), np.concatenate(rules)


@pytest.mark.parametrize("W", [1, 2, 3, 8])
def test_merge_rank_runs_numpy(W):
    rng = np.random.default_rng(700 + W)
    N = 50
    rb, t, r = _runs(rng, N, W)
    tt, rr = torch.from_numpy(t.copy()), torch.from_numpy(r.copy())
    shard.merge_rank_runs(rb, tt, rr)
    for n in range(N):
        a, b = rb[n, 0], rb[n, -1]
        o = np.lexsort((r[a:b], t[a:b]))
        if W == 1:
            o = np.arange(b - a)  # one run: already in order, untouched
        assert np.array_equal(tt.numpy()[a:b], t[a:b][o]), n
        assert np.array_equal(rr.numpy()[a:b], r[a:b][o]), n
