"""Schedule.Next on the GPU (cg_next_batch) vs the reference's KATs and the
oracle's literal Go walk, bit-exact."""
import json
import os

import zlib

import numpy as np
import pytest

import oracle_lib as O
from common import ZONES, oracle_zone, product_zone, random_spec

pytestmark = pytest.mark.gpu

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kats.json")))


@pytest.fixture(scope="module")
def eng():
    from cronsun_amd.engine import Engine
    return Engine(0)


def _zone(name):
    return product_zone(name)


def test_kats_next_and_activation(eng):
    from cronsun_amd import cron
    rows = KATS["next"] + KATS["next_tz"]
    by_zone = {}
    for r in rows:
        by_zone.setdefault(r["zone"], []).append((r["spec"], r["time"], r["expected"], r["ref"]))
    for r in KATS["activation"]:
        by_zone.setdefault(r["zone"], []).append((r["spec"], r["time"] - 1, r, r["ref"]))
    n = 0
    for zone, items in by_zone.items():
        z = _zone(zone)
        scheds = [cron.Parse(s) for s, _, _, _ in items]
        t = np.array([t for _, t, _, _ in items], dtype=np.int64)
        got = eng.next_batch(scheds, z, t)
        for (s, t_in, exp, ref), g in zip(items, got):
            if isinstance(exp, dict):  # TestActivation: Next(t-1s) == t iff expected
                assert (int(g) == exp["time"]) == exp["expected"], ref
            else:
                assert int(g) == exp, (ref, s, int(g), exp)
            n += 1
    assert n == 74


def test_kat_constant_delay(eng):
    from cronsun_amd import cron
    rows = [r for r in KATS["constant_delay"] if r["nsec"] == 0]
    scheds = [cron.Every(r["delay_ns"]) for r in rows]
    got = eng.next_batch(scheds, None, np.array([r["time"] for r in rows], dtype=np.int64))
    assert [int(x) for x in got] == [r["expected"] for r in rows]


def test_schedule_next_method():
    from cronsun_amd import cron
    ny = _zone("America/New_York")
    s = cron.Parse("0 0 1 * * ?")
    assert s.Next(1352005200, ny) == 1352008800  # 2012-11-04 01:00 EDT -> 01:00 EST


@pytest.mark.parametrize("zone", ZONES)
def test_random_specs_vs_oracle(eng, zone):
    from cronsun_amd import cron
    rng = np.random.default_rng(zlib.crc32(zone.encode()))
    n = 1500
    specs = [random_spec(rng) for _ in range(n)]
    scheds = [cron.Parse(s) for s in specs]
    # instants across 2000-2040, a third of them within a day of a transition
    t = rng.integers(946684800, 2208988800, n)
    from test_zone import _table
    when, _ = _table(z := _zone(zone), 946684800, 2208988800)
    if len(when) > 1:
        near = rng.integers(0, n, n // 3)
        t[near] = when[rng.integers(1, len(when), len(near))] + rng.integers(-86400, 86400, len(near))
    got = eng.next_batch(scheds, z, t)
    oz = oracle_zone(zone)
    for i in range(n):
        osched, err = O.parse(specs[i])  # the oracle's own parser, not the product's masks
        assert err is None, (specs[i], err)
        exp = O.sched_next(osched, int(t[i]), oz)
        assert int(got[i]) == exp, (zone, specs[i], int(t[i]), int(got[i]), exp)


def test_never_fires_returns_zero_time(eng):
    from cronsun_amd import cron
    scheds = [cron.Parse("0 0 0 30 Feb ?"), cron.Parse("0 0 0 31 Apr ?"),
              cron.Parse("0 0 0 , * *"), cron.Parse("0 0 0 31 Feb,Apr ?")]
    got = eng.next_batch(scheds, None, np.full(4, 1341878400, dtype=np.int64))
    assert all(int(x) == cron.ZERO_TIME if hasattr(cron, "ZERO_TIME") else int(x) == -62135596800
               for x in got)
