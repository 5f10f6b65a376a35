"""The GPU-resident dispatcher (cg_dispatcher_*) against the oracle's Cron.run
wake loop (or_cron_*), wake by wake: the effective time, the set of entries
fired and every entry's Next/Prev, bit-exact, with adds and removes while
running and late wakes that skip missed fires.  Then the Cron mirror
(cronsun_amd.dispatch) through node/cron/cron_test.go's wall-clock cases."""
import threading
import time
import zlib

import numpy as np
import pytest

import oracle_lib as O
from common import oracle_parse_all, oracle_zone, product_zone, random_spec

pytestmark = pytest.mark.gpu

Z = O.ZERO_TIME


@pytest.fixture(scope="module")
def eng():
    from cronsun_amd.engine import Engine
    return Engine(0)


def _check_snapshot(d, oc):
    nx, pv, live = d.snapshot()
    snap = oc.snapshot()
    for i in range(len(nx)):
        if i in snap:
            assert live[i] and (int(nx[i]), int(pv[i])) == snap[i], (i, int(nx[i]), int(pv[i]), snap[i])
        else:
            assert not live[i]


# zones without skipped local days (where the reference Next never returns)
@pytest.mark.parametrize("zone,t0", [
    ("UTC", 1767225600),
    ("America/New_York", 1772953200 - 5400),    # 90 min before 2026-03-08 02:00 EST
    ("Australia/Lord_Howe", 1775314800 - 3600),  # before the 30-minute fall-back
    ("Europe/London", 1792890000 - 3600),
    ("Asia/Kathmandu", 1767225600),
])
def test_dispatcher_vs_oracle(eng, zone, t0):
    from cronsun_amd import cron
    rng = np.random.default_rng(zlib.crc32(b"dispatch" + zone.encode()))
    n = 1500
    specs = [random_spec(rng) for _ in range(n)]
    scheds = [cron.Parse(s) for s in specs]
    osch = oracle_parse_all(specs)  # the oracle's own parser
    oc = O.OracleCron(osch, oracle_zone(zone))
    z = product_zone(zone)
    oc.start(t0)
    d = eng.dispatcher(scheds, z, t0)
    _check_snapshot(d, oc)
    next_slot = n
    for w in range(120):
        e = oc.effective()
        assert d.effective == e, w
        if e == Z:
            break
        late = int(rng.choice([0, 0, 0, 1, 2, 59, 700, 4000]))
        now = e + late
        due, e2 = d.fire(now)
        assert [int(x) for x in due] == oc.fire(e, now), (w, e, now)
        assert e2 == oc.effective()
        if w % 15 == 7:  # add / replace / remove while running
            k = int(rng.integers(1, 6))
            slots = [int(x) for x in rng.choice(next_slot, k, replace=False)]
            if rng.random() < 0.5:
                slots.append(next_slot)
                next_slot += 1
            new_specs = [random_spec(rng) for _ in slots]
            new = [cron.Parse(x) for x in new_specs]
            d.set(slots, new, now)
            for s, osc in zip(slots, oracle_parse_all(new_specs)):
                oc.set(s, osc, now)
            rm = [int(x) for x in rng.choice(n, 3, replace=False) if int(x) not in slots]
            d.remove(rm)
            for s in rm:
                oc.remove(s)
        if w % 40 == 39:
            _check_snapshot(d, oc)
    _check_snapshot(d, oc)
    d.free()


def test_dispatcher_many_equal_due(eng):
    """A wake that fires most of a large table at once: the due list is the
    ascending slot list and the tile compaction covers every tile."""
    from cronsun_amd import cron
    n = 3 * 4096 + 123
    scheds = [cron.Every(60 * 10**9) if i % 7 else cron.Parse("0 0 * * * *") for i in range(n)]
    t0 = 1767225600
    d = eng.dispatcher(scheds, None, t0)
    assert d.effective == t0 + 60
    due, e2 = d.fire(t0 + 60)
    assert np.array_equal(due, np.array([i for i in range(n) if i % 7], dtype=np.int32))
    assert e2 == t0 + 120
    nx, pv, _ = d.snapshot()
    assert int(nx[1]) == t0 + 120 and int(pv[1]) == t0 + 60 and int(pv[0]) == Z
    d.free()


def test_dispatcher_empty_and_never(eng):
    from cronsun_amd import cron
    d = eng.dispatcher([cron.Parse("0 0 0 30 Feb ?")], None, 1767225600)
    assert d.effective == Z
    assert d.fire(1767225600 + 10)[0].size == 0
    d.set([5], [cron.Parse("@every 5s")], 1767225600)
    assert len(d) == 6 and d.effective == 1767225605
    nx, pv, live = d.snapshot()
    assert list(live) == [True, False, False, False, False, True]
    d.remove([5])
    assert d.effective == Z
    d.free()


# ------------------------------------------------ cron_test.go, wall clock
ONE_SECOND = 1.25  # cron_test.go:15 uses 1.01 s; a little slack for Python threads


class WG:
    """sync.WaitGroup"""

    def __init__(self, n):
        self.n = n
        self.cv = threading.Condition()

    def Done(self):
        with self.cv:
            self.n -= 1
            self.cv.notify_all()

    def wait(self, timeout):
        with self.cv:
            return self.cv.wait_for(lambda: self.n <= 0, timeout)


class NamedJob:
    """cron_test.go:280-291 testJob"""

    def __init__(self, wg, name):
        self.wg, self.name = wg, name

    def GetID(self):
        return self.name

    def Run(self):
        self.wg.Done()


def _boom():
    raise RuntimeError("YOLO")


def test_func_panic_recovery(eng):
    from cronsun_amd.dispatch import Cron
    c = Cron(engine=eng)
    c.Start()
    c.AddFunc("* * * * * ?", _boom)
    time.sleep(ONE_SECOND)
    c.Stop()


def test_no_entries_and_stop_without_start(eng):
    from cronsun_amd.dispatch import Cron
    Cron(engine=eng).Stop()
    c = Cron(engine=eng)
    c.Start()
    t = time.time()
    c.Stop()
    assert time.time() - t < ONE_SECOND


def test_stop_causes_jobs_to_not_run(eng):
    from cronsun_amd.dispatch import Cron
    wg = WG(1)
    c = Cron(engine=eng)
    c.Start()
    c.Stop()
    c.AddFunc("* * * * * ?", wg.Done)
    assert not wg.wait(ONE_SECOND)


def test_add_before_and_while_running(eng):
    from cronsun_amd.dispatch import Cron
    wg = WG(1)
    c = Cron(engine=eng)
    c.AddFunc("* * * * * ?", wg.Done)
    c.Start()
    assert wg.wait(ONE_SECOND)
    c.Stop()
    wg = WG(1)
    c = Cron(engine=eng)
    c.Start()
    c.AddFunc("* * * * * ?", wg.Done)
    assert wg.wait(ONE_SECOND)
    c.Stop()


def test_add_while_running_with_delay(eng):
    from cronsun_amd.dispatch import Cron
    c = Cron(engine=eng)
    c.Start()
    time.sleep(2)  # cron_test.go:123 sleeps 5 s
    calls = []
    c.AddFunc("* * * * * *", lambda: calls.append(1))
    time.sleep(1.01)
    c.Stop()
    assert len(calls) == 1


def test_snapshot_entries(eng):
    from cronsun_amd.dispatch import Cron
    wg = WG(1)
    c = Cron(engine=eng)
    c.AddFunc("@every 2s", wg.Done)
    c.Start()
    time.sleep(1.01)
    c.Entries()
    assert wg.wait(ONE_SECOND)
    c.Stop()


def test_multiple_entries_and_schedules(eng):
    from cronsun_amd import cron
    from cronsun_amd.dispatch import Cron, FuncJob
    wg = WG(4)
    c = Cron(engine=eng)
    c.AddFunc("0 0 0 1 1 ?", lambda: None)
    c.AddFunc("* * * * * ?", wg.Done)
    c.AddFunc("0 0 0 31 12 ?", lambda: None)
    f2 = lambda: wg.Done()  # noqa: E731
    c.AddFunc("* * * * * ?", f2)
    c.Schedule(cron.Every(60 * 10**9), FuncJob(lambda: None))
    f3 = lambda: wg.Done()  # noqa: E731
    c.Schedule(cron.Every(10**9), FuncJob(f3))
    c.Start()
    assert wg.wait(2 * ONE_SECOND)
    c.Stop()


def test_non_local_timezone(eng):
    from cronsun_amd import cron
    from cronsun_amd.dispatch import Cron
    loc = cron.FixedZone("Atlantic/Cape_Verde", -3600)  # cron_test.go:247-271
    wg = WG(2)
    lt = time.gmtime(int(time.time()) - 3600)
    if lt.tm_sec >= 57:  # keep both seconds inside this minute
        time.sleep(4)
        lt = time.gmtime(int(time.time()) - 3600)
    spec = f"{lt.tm_sec + 1},{lt.tm_sec + 2} {lt.tm_min} {lt.tm_hour} {lt.tm_mday} {lt.tm_mon} ?"
    c = Cron(loc, engine=eng)
    c.AddFunc(spec, wg.Done)
    c.Start()
    assert wg.wait(2 * ONE_SECOND), spec
    c.Stop()


def test_job_order(eng):
    from cronsun_amd import cron
    from cronsun_amd.dispatch import Cron
    wg = WG(1)
    c = Cron(engine=eng)
    c.AddJob("0 0 0 30 Feb ?", NamedJob(wg, "job0"))
    c.AddJob("0 0 0 1 1 ?", NamedJob(wg, "job1"))
    c.AddJob("* * * * * ?", NamedJob(wg, "job2"))
    c.AddJob("1 0 0 1 1 ?", NamedJob(wg, "job3"))
    c.Schedule(cron.Every(5 * 10**9 + 5), NamedJob(wg, "job4"))
    c.Schedule(cron.Every(5 * 60 * 10**9), NamedJob(wg, "job5"))
    c.Start()
    assert wg.wait(ONE_SECOND)
    assert [e.Job.name for e in c.Entries()] == ["job2", "job4", "job5", "job1", "job3", "job0"]
    c.Stop()
