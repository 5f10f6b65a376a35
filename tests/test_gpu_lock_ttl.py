"""Batch Cmd.lockTtl on the GPU (cg_lock_ttl_batch / k_lock_ttl) against the
oracle's restatement of job.go:194-233, bit-exact, over random specs, zones,
instants near transitions, job kinds, AvgTimes (including negative and
extreme values, where Go's int64 arithmetic wraps) and LockTtl values."""
import zlib

import numpy as np
import pytest

import oracle_lib as O
from common import oracle_parse_all, oracle_zone, product_zone, random_spec

pytestmark = pytest.mark.gpu

AVGS = [0, 999, 1000, 1500, 3500, -1, -999, -2500, 3_600_000, -(1 << 63), (1 << 63) - 1]


@pytest.fixture(scope="module")
def eng():
    from cronsun_amd.engine import Engine
    return Engine(0)


@pytest.mark.parametrize("zone", ["UTC", "America/New_York", "Pacific/Apia", "Australia/Lord_Howe",
                                  "Africa/Casablanca", "fixed:19800"])
def test_lock_ttl_vs_oracle(eng, zone):
    from cronsun_amd import cron
    rng = np.random.default_rng(zlib.crc32(b"lockttl" + zone.encode()))
    n = 1200
    specs = [random_spec(rng) for _ in range(n)]
    scheds = [cron.Parse(s) for s in specs]
    now = rng.integers(946684800, 2208988800, n)
    from test_zone import _table
    z = product_zone(zone)
    when, _ = _table(z, 946684800, 2208988800)
    if len(when) > 1:
        near = rng.integers(0, n, n // 3)
        now[near] = when[rng.integers(1, len(when), len(near))] + rng.integers(-86400, 86400, len(near))
    kind = rng.integers(0, 4, n).astype(np.int32)  # 3: an unknown kind takes the common path
    avg = rng.integers(-5000, 20000, n)
    pick = rng.integers(0, n, n // 5)
    avg[pick] = np.array(AVGS, dtype=np.int64)[rng.integers(0, len(AVGS), len(pick))]
    oz = oracle_zone(zone)
    osch = oracle_parse_all(specs)  # the oracle's own parser
    sp = eng.upload(scheds)
    for L in (300, 2, 86400):
        got = eng.lock_ttl_batch(sp, z, now, kind, avg, L)
        for i in range(n):
            exp = O.lock_ttl(osch[i], int(now[i]), oz, int(kind[i]), int(avg[i]), L)
            assert int(got[i]) == exp, (zone, specs[i], int(now[i]), int(kind[i]), int(avg[i]), L,
                                        int(got[i]), exp)


def test_lock_ttl_never_fires_and_scalar_args(eng):
    from cronsun_amd import cron
    scheds = [cron.Parse("0 0 0 30 Feb ?"), cron.Parse("@every 10s"), cron.Parse("@every 1s"),
              cron.Parse("0 */5 * * * *")]
    got = eng.lock_ttl_batch(scheds, None, 1767225600, 0, 1000, 1000)
    assert [int(x) for x in got] == [0, 9, 2, 299]
    got = eng.lock_ttl_batch(scheds, None, 1767225600, 2, 1000, 1000)
    assert [int(x) for x in got] == [0, 8, 1, 298]


def test_jobset_lock_ttls(eng):
    from cronsun_amd.model import Job, JobRule, JobSet, KindInterval
    jobs = [Job("a", Rules=[JobRule("r1", "@every 30s"), JobRule("r2", "0 0 * * * *")], AvgTime=4200),
            Job("b", Kind=KindInterval, Rules=[JobRule("r3", "@every 30s")])]
    js = JobSet(jobs, {})
    assert [int(x) for x in js.lock_ttls(1767225600, engine=eng)] == [26, 300, 28]
