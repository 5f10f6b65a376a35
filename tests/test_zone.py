"""Host zone rules (TZif + POSIX footer, cg_zone_*) and the flat breakpoint
table the kernels use, against the oracle's literal Location.lookup."""
import ctypes as C

import numpy as np
import pytest

from common import ZONES, oracle_zone, product_zone
from cronsun_amd import _lib


def _table(z, lo, hi):
    L = _lib.lib()
    n = L.cg_zone_table(z.handle, lo, hi, None, None, 0)
    when = np.zeros(n, dtype=np.int64)
    off = np.zeros(n, dtype=np.int32)
    L.cg_zone_table(z.handle, lo, hi, when.ctypes.data, off.ctypes.data, n)
    return when, off


def _probe_times(rng, lo, hi, n=4000):
    t = rng.integers(lo, hi, n)
    return np.concatenate([t, [lo, hi]])


@pytest.mark.parametrize("name", ZONES)
def test_offsets_match_oracle(name):
    z, oz = product_zone(name), oracle_zone(name)
    rng = np.random.default_rng(1)
    for t in _probe_times(rng, -2208988800, 4102444800, 3000):  # 1900..2100
        assert z.offset(int(t)) == oz.lookup(int(t))[0], (name, int(t))


@pytest.mark.parametrize("name", ZONES)
@pytest.mark.parametrize("span", [(1577836800, 1893456000), (0, 86400 * 400), (-1000000000, -900000000)])
def test_breakpoint_table_matches_oracle(name, span):
    lo, hi = span
    z, oz = product_zone(name), oracle_zone(name)
    when, off = _table(z, lo, hi)
    assert when[0] == np.iinfo(np.int64).min
    assert (when[2:] > when[1:-1]).all()
    assert (off[1:] != off[:-1]).all()
    rng = np.random.default_rng(2)
    probes = list(_probe_times(rng, lo, hi, 2000))
    for w in when[1:]:  # both sides of every breakpoint
        probes += [int(w) - 1, int(w), int(w) + 1]
    for t in probes:
        t = int(t)
        if t < lo or t > hi:
            continue
        i = np.searchsorted(when, t, side="right") - 1
        assert off[i] == oz.lookup(t)[0], (name, t)


def test_new_york_footer_expanded():
    # 2026 NY transitions come from the TZif footer EST5EDT,M3.2.0,M11.1.0
    z = product_zone("America/New_York")
    when, off = _table(z, 1767225600, 1798761600)  # 2026
    assert list(when[1:]) == [1772953200, 1793512800]  # Mar 8 07:00Z, Nov 1 06:00Z
    assert list(off) == [-18000, -14400, -18000]


def test_fixed_and_utc():
    assert product_zone("UTC").offset(123) == 0
    assert product_zone("fixed:19800").offset(-10**12) == 19800
