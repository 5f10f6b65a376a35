"""Cmd.lockTtl (job.go:194-233), CPU side: the oracle's restatement against
known answers derived by hand from job.go, and the batch algorithm the
k_lock_ttl kernel runs (next_exact twice + lock_ttl_of, compiled for the
host, tests/native/lock_ttl_host.cpp) against the oracle on random specs,
kinds, AvgTimes and LockTtl values.  The reference has no test for lockTtl;
these answers follow job.go's statements, so parity here is pinned to the
oracle's Next (itself pinned by spec_test.go's KATs) plus the arithmetic."""
import os
import subprocess

import pytest

import oracle_lib as O
from common import oracle_zone

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON, ALONE, INTERVAL = 0, 1, 2
T2026 = 1767225600  # 2026-01-01 00:00:00 UTC


def _ttl(spec, kind, avg, L=300, zone="UTC", now=T2026, nsec=0):
    s, err = O.parse(spec)
    assert err is None, err
    return O.lock_ttl(s, now, oracle_zone(zone), kind, avg, L, nsec=nsec)


@pytest.mark.parametrize("spec,kind,avg,L,exp", [
    ("@every 10s", COMMON, 0, 300, 10),
    ("@every 10s", ALONE, 3500, 300, 7),      # cost = 3500/1e3 = 3, no round-up
    ("@every 10s", COMMON, 999, 300, 10),     # cost 0
    ("@every 10s", COMMON, 12000, 300, 10),   # ttl < cost: unchanged
    ("@every 10s", COMMON, -2500, 300, 11),   # cost -2, "round-up" -> -1
    ("@every 10s", INTERVAL, 3500, 300, 8),   # ttl - 2
    ("@every 1s", INTERVAL, 0, 300, 1),       # clamp to >= 1
    ("@every 1s", COMMON, 0, 300, 2),         # clamp to >= 2
    ("@every 1h", COMMON, 0, 300, 300),       # LockTtl cap
    ("@every 1h", INTERVAL, 0, 300, 300),
    ("@every 1h", COMMON, 60000, 10000, 3540),
    ("@every 1h", INTERVAL, 60000, 10000, 3598),
    ("@hourly", ALONE, 0, 300, 300),
    ("0 */5 * * * *", ALONE, 1000, 1000, 299),
    ("0 0 0 30 2 *", COMMON, 0, 300, 0),      # never fires: ttl 0 (lock() refuses it)
    ("0 0 0 30 2 *", INTERVAL, 0, 300, 0),
])
def test_lock_ttl_kats(spec, kind, avg, L, exp):
    assert _ttl(spec, kind, avg, L) == exp


def test_lock_ttl_across_dst():
    ny = oracle_zone("America/New_York")
    L = O.lib()
    # @daily from Saturday noon: the next two midnights straddle the spring-forward
    # (23 h) and fall-back (25 h) Sundays of 2026
    spring = L.or_date(2026, 3, 7, 12, 0, 0, ny.h)
    fall = L.or_date(2026, 10, 31, 12, 0, 0, ny.h)
    assert _ttl("@daily", COMMON, 0, 10 ** 6, "America/New_York", spring) == 23 * 3600
    assert _ttl("@daily", COMMON, 0, 10 ** 6, "America/New_York", fall) == 25 * 3600


def test_lock_ttl_nanoseconds_of_now_dropped():
    # Next truncates now's nanoseconds (spec.go:61, constantdelay.go:26)
    assert _ttl("@every 10s", COMMON, 0, nsec=999_999_999) == 10
    assert _ttl("*/7 * * * * *", COMMON, 0, nsec=500) == _ttl("*/7 * * * * *", COMMON, 0)


@pytest.fixture(scope="module")
def lock_ttl_host():
    O.lib()
    src = os.path.join(ROOT, "tests", "native", "lock_ttl_host.cpp")
    out = os.path.join(ROOT, "tests", "native", "lock_ttl_host")
    deps = [src, os.path.join(ROOT, "tests", "native", "host_common.h"),
            os.path.join(ROOT, "cronsun_amd", "csrc", "cg_time.h"),
            os.path.join(ROOT, "cronsun_amd", "csrc", "cg_zone.cpp")]
    if not os.path.exists(out) or any(os.path.getmtime(out) < os.path.getmtime(d) for d in deps):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", out, src, deps[-1],
                               "-L" + os.path.join(ROOT, "oracle"), "-loracle",
                               "-Wl,-rpath," + os.path.join(ROOT, "oracle")])
    return out


@pytest.mark.parametrize("zone", ["UTC", "America/New_York", "Pacific/Apia", "Australia/Lord_Howe",
                                  "Europe/London", "Asia/Kathmandu"])
def test_batch_algorithm_matches_oracle(lock_ttl_host, zone):
    out = subprocess.run([lock_ttl_host, zone, "2500", "5"], cwd=ROOT, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert " 0 mismatches" in out.stdout
