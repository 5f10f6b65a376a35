"""Cron.run (node/cron/cron.go:210-275), CPU side: the oracle's wake loop
(or_cron_*: byTime sort, the due prefix, Next(now) for each fired entry)
against answers derived by hand from cron.go, and the host bookkeeping of the
Cron mirror (cronsun_amd.dispatch) before Start.  The GPU dispatcher is checked
against this oracle in tests/test_gpu_dispatch.py.  The reference's own
cron_test.go cases that need wall-clock goroutines are covered there."""
import oracle_lib as O
from common import oracle_zone

T0 = 1767225600  # 2026-01-01 00:00:00 UTC
Z = O.ZERO_TIME


def _oc(specs, zone="UTC"):
    scheds = []
    for sp in specs:
        s, err = O.parse(sp)
        assert err is None, err
        scheds.append(s)
    return O.OracleCron(scheds, oracle_zone(zone))


def test_oracle_wake_sequence():
    c = _oc(["@every 10s", "*/5 * * * * *", "0 0 0 30 2 *"])
    c.start(T0)
    assert c.snapshot() == {0: (T0 + 10, Z), 1: (T0 + 5, Z), 2: (Z, Z)}
    e = c.effective()
    assert e == T0 + 5
    assert c.fire(e, e) == [1]
    e = c.effective()
    assert e == T0 + 10
    assert c.fire(e, e) == [0, 1]            # equal Next values fire together
    assert c.snapshot()[0] == (T0 + 20, T0 + 10)
    e = c.effective()
    assert e == T0 + 15
    assert c.fire(e, T0 + 47) == [1]          # a late wake: Next(now) skips missed fires
    assert c.snapshot()[1] == (T0 + 50, T0 + 15)
    assert c.effective() == T0 + 20


def test_oracle_zero_sorts_last_and_empty():
    c = _oc(["0 0 0 30 2 *", "0 0 0 31 4 *"])
    c.start(T0)
    assert c.effective() == Z                 # the loop sleeps ten years
    assert _oc([]).effective() == Z


def test_oracle_add_and_remove():
    c = _oc(["@every 1h"])
    c.start(T0)
    s, _ = O.parse("@every 30s")
    c.set(1, s, T0 + 7)                       # added while running: Next(time.Now())
    assert c.effective() == T0 + 37
    c.remove(1)
    assert c.effective() == T0 + 3600


def test_cron_mirror_bookkeeping_before_start():
    from cronsun_amd.dispatch import Cron, FuncJob
    c = Cron()
    hits = []
    f = lambda: hits.append(1)  # noqa: E731
    c.AddFunc("@every 1s", f)
    c.AddFunc("0 0 * * * *", f)               # same func: same ID, replaced in place
    assert len(c.Entries()) == 1
    assert c.Entries()[0].ID == FuncJob(f).GetID()
    c.DelFunc(f)
    assert c.Entries() == []
    try:
        c.AddFunc("bad spec here", f)
        raise AssertionError("parse error expected")
    except ValueError:
        pass
