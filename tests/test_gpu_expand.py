"""Batch expansion on the GPU (cg_expand*) vs the oracle's literal Next loop:
t = T0; loop { t = Next(t); if t.IsZero() || t > T1 break; emit t }.
Bit-exact CSR (offsets and times) on seeded inputs; size-independent
properties at the BASELINE config-2 scale."""
import zlib

import numpy as np
import pytest

import oracle_lib as O
from common import ZONES, oracle_parse_all, oracle_zone, product_zone, random_spec, to_oracle_sched
from cronsun_amd import _lib, cron, synth

pytestmark = pytest.mark.gpu

DAY = 86400


@pytest.fixture(scope="module")
def eng():
    from cronsun_amd.engine import Engine
    return Engine(0)


def oracle_csr(scheds, zone, t0, t1, specs=None):
    """The oracle's Next loop; with the spec strings it parses them with its
    own parser (parser.go restated), so the product parser is checked too."""
    if specs is not None:
        arr = O.sched_array(oracle_parse_all(specs))
    else:
        arr = O.sched_array([to_oracle_sched(s.to_c()) for s in scheds])
    return O.expand_batch(arr, t0, t1, oracle_zone(zone), threads=8)


def check_same(eng, scheds, zone, t0, t1, specs=None):
    try:
        eo, et = oracle_csr(scheds, zone, t0, t1, specs)
    except O.NonTerminating as e:
        # the reference loop cycles for these rules: the engine must refuse the
        # batch with CG_ERANGE, and agree with the oracle on every other rule
        with pytest.raises(_lib.CgError) as err:
            eng.expand(scheds, product_zone(zone), t0, t1)
        assert err.value.code == _lib.CG_ERANGE
        assert f"rule {e.rules[0]}:" in err.value.msg
        keep = [i for i in range(len(scheds)) if i not in set(e.rules)]
        return check_same(eng, [scheds[i] for i in keep], zone, t0, t1,
                          [specs[i] for i in keep] if specs else None)
    off, times = eng.expand(scheds, product_zone(zone), t0, t1)
    if not np.array_equal(off, eo):
        bad = np.nonzero(np.diff(off) != np.diff(eo))[0][:5]
        msg = [(specs[i] if specs else i, int(off[i + 1] - off[i]), int(eo[i + 1] - eo[i])) for i in bad]
        raise AssertionError(f"counts differ {zone} ({t0},{t1}]: {msg}")
    if not np.array_equal(times, et):
        i = int(np.nonzero(times != et)[0][0])
        r = int(np.searchsorted(off, i, side="right") - 1)
        raise AssertionError(f"times differ {zone} rule {specs[r] if specs else r} idx {i}: "
                             f"{int(times[i])} vs {int(et[i])}")
    return off, times


def _horizons(zone):
    from test_zone import _table
    z = product_zone(zone)
    when, _ = _table(z, 1735689600, 1830297600)  # 2025..2027
    hs = [(synth.T0_2026, synth.T0_2026 + 3600), (synth.T0_2026 + 1234, synth.T0_2026 + DAY)]
    for w in when[1:5]:
        w = int(w)
        hs.append((w - DAY // 2 - 17, w + DAY // 2))          # straddles a transition
        hs.append((w - 3 * DAY, w + 4 * DAY))                  # 7 days around it
    return hs


@pytest.mark.parametrize("zone", ZONES)
def test_random_specs_vs_oracle(eng, zone):
    rng = np.random.default_rng(zlib.crc32(("x" + zone).encode()))
    specs = [random_spec(rng) for _ in range(300)]
    scheds = [cron.Parse(s) for s in specs]
    for t0, t1 in _horizons(zone):
        check_same(eng, scheds, zone, t0, t1, specs)


@pytest.mark.parametrize("zone", ["UTC", "America/New_York", "Australia/Lord_Howe"])
def test_synthetic_mix_vs_oracle(eng, zone):
    specs = synth.spec_mix(2000, seed=3)
    scheds = [cron.Parse(s) for s in specs]
    check_same(eng, scheds, zone, synth.T0_2026, synth.T0_2026 + DAY, specs)
    ny_spring = 1772953200  # 2026-03-08T07:00Z
    check_same(eng, scheds, zone, ny_spring - 6 * 3600, ny_spring + 6 * 3600, specs)


def test_long_horizon_multi_chunk(eng):
    # > 30 days: several closed-form chunks, each re-anchored by an exact Next
    rng = np.random.default_rng(5)
    specs = ["0 0 9 * * 1-5", "0 0 0 29 Feb ?", "0 15 10 15 * ?", "@weekly", "@monthly",
             "0 0 0 1 Jan,Jul ?", "0 0 12 * * Sun", "@every 6h", "0 30 2 * * *", "@daily"]
    specs += [random_spec(rng) for _ in range(40) if True]
    specs = [s for s in specs if not s.startswith("@every") or True]
    scheds = [cron.Parse(s) for s in specs]
    for zone in ("UTC", "America/New_York", "Australia/Sydney", "America/Havana"):
        check_same(eng, scheds, zone, synth.T0_2026 - 17, synth.T0_2026 + 100 * DAY, specs)


def test_edge_cases(eng):
    scheds = [cron.Parse(s) for s in ["0 0 0 30 Feb ?", "* * * * * *", "@every 1s", "0 0 0 * * *"]]
    z = product_zone("UTC")
    # empty horizon and reversed horizon
    off, times = eng.expand(scheds, z, synth.T0_2026, synth.T0_2026)
    assert off.tolist() == [0, 0, 0, 0, 0] and times.size == 0
    off, times = eng.expand(scheds, z, synth.T0_2026, synth.T0_2026 - 5)
    assert off[-1] == 0
    # one second horizon: the every-second spec and @every 1s fire once
    off, times = eng.expand(scheds, z, synth.T0_2026, synth.T0_2026 + 1)
    assert off.tolist() == [0, 0, 1, 2, 2]
    # empty rule set
    off, times = eng.expand([], z, 0, 100)
    assert off.tolist() == [0] and times.size == 0
    # the horizon limit (40 years) is enforced
    with pytest.raises(_lib.CgError) as e:
        eng.expand(scheds, z, 0, _lib.MAX_HORIZON + 1)
    assert e.value.code == _lib.CG_ERANGE


LONG_SPECS = ["@yearly", "@monthly", "@weekly", "@daily", "0 0 0 29 Feb ?", "59 59 23 28,29 Feb ?",
              "0 0 12 29 Feb Mon", "0 30 2 * * *", "0 30 1 * * Sun", "0 0 0 31 * ?", "0 0 0 30 Feb ?",
              "0 15 10 15 * ?", "0 0 9 * * 1-5", "0 0 */6 1 Jan,Jul *", "@every 7h", "@every 90000s",
              "30 59 23 31 Dec ?", "0 0 0 1 Jan ?"]


@pytest.mark.parametrize("zone", ["UTC", "America/New_York", "Australia/Lord_Howe"])
def test_multi_year_horizons(eng, zone):
    """Horizons past one year (spec.go:70-76): three years from 2026, and
    2095-06-01 .. 2106-06-01 where Feb 29 skips 2100, so Next's five-year
    limit returns the zero time after 2096-02-29 and ends that rule's loop."""
    rng = np.random.default_rng(zlib.crc32(("long" + zone).encode()))
    specs = list(LONG_SPECS)
    while len(specs) < 60:  # sparse random specs: at most one fire per matching hour
        f = random_spec(rng).split(" ")
        if len(f) >= 5 and not f[0].startswith("@"):
            specs.append(" ".join([str(rng.integers(0, 60)), str(rng.integers(0, 60))] + f[2:]))
    scheds = [cron.Parse(s) for s in specs]
    off, _ = check_same(eng, scheds, zone, synth.T0_2026 - 77, synth.T0_2026 + 1096 * DAY, specs)
    assert off[-1] > 10_000
    off, times = check_same(eng, scheds, zone, 3957984000, 3957984000 + 4018 * DAY, specs)
    feb29 = specs.index("0 0 0 29 Feb ?")
    assert off[feb29 + 1] - off[feb29] == 1  # 2096-02-29 only: 2104 is past the limit


def test_feb29_across_leap_years(eng):
    specs = ["0 0 0 29 Feb ?", "59 59 23 28,29 Feb ?"]
    scheds = [cron.Parse(s) for s in specs]
    t0 = 1704067200  # 2024-01-01
    check_same(eng, scheds, "UTC", t0, t0 + 365 * DAY, specs)
    check_same(eng, scheds, "America/New_York", t0 + 40 * DAY, t0 + 70 * DAY, specs)


def test_config2_scale_properties(eng):
    """BASELINE config 2 (1M mixed rules x 24 h, UTC) at full size: the
    size-independent invariants, plus bit-exact rows on a seeded sample."""
    n = 1_000_000
    specs = synth.spec_mix(n, seed=0x5EED)
    arr, status = cron.parse_batch(specs)
    assert (status == 0).all()
    sp = eng.upload_c(arr, n)
    t0, t1 = synth.T0_2026, synth.T0_2026 + DAY
    E = eng.expand_device(sp, None, t0, t1)
    off = np.empty(n + 1, dtype=np.int64)
    from cronsun_amd._lib import check, lib
    check(lib().cg_result_copy_offsets(eng._h, off.ctypes.data))
    assert off[0] == 0 and off[-1] == E and (np.diff(off) >= 0).all()
    times = eng.copy_times(0, E)
    assert ((times > t0) & (times <= t1)).all()
    # strictly increasing inside every rule: the only non-increasing steps are at rule starts
    steps = np.nonzero(np.diff(times) <= 0)[0] + 1
    assert np.isin(steps, off[1:-1]).all()
    # bit-exact on a seeded sample of rules
    rng = np.random.default_rng(9)
    idx = np.sort(rng.choice(n, 3000, replace=False))
    sample = [cron.Parse(specs[i]) for i in idx]
    eo, et = oracle_csr(sample, "UTC", t0, t1, [specs[i] for i in idx])
    for k, i in enumerate(idx):
        got = times[off[i]:off[i + 1]]
        exp = et[eo[k]:eo[k + 1]]
        assert np.array_equal(got, exp), specs[i]


def test_plan_cache_survives_other_entry_points(eng):
    """Next/lockTtl upload their own zone tables into the context's plan
    buffer: a repeated expansion over the same (zone, T0, T1) must rebuild its
    plan rather than reuse the cached one."""
    rng = np.random.default_rng(11)
    scheds = [cron.Parse(random_spec(rng)) for _ in range(400)]
    ny = product_zone("America/New_York")
    t0 = 1772900000
    sp = eng.upload(scheds)
    first = eng.expand(sp, ny, t0, t0 + 3 * DAY)
    eng.next_batch(sp, product_zone("Australia/Lord_Howe"), np.full(len(scheds), t0, dtype=np.int64))
    eng.lock_ttl_batch(sp, product_zone("Pacific/Apia"), t0, 0, 0)
    again = eng.expand(sp, ny, t0, t0 + 3 * DAY)
    assert np.array_equal(first[0], again[0]) and np.array_equal(first[1], again[1])


def test_lean_phase_timing_same_result(eng):
    """cg_set_phase_timing(1) drops the events between phases (throughput
    runs): the result is unchanged, k_write_cf is still timed and the
    untimed phases read -1."""
    rng = np.random.default_rng(12)
    scheds = [cron.Parse(random_spec(rng)) for _ in range(2000)]
    sp = eng.upload(scheds)
    ny = product_zone("America/New_York")
    t0 = 1772900000
    full = eng.expand(sp, ny, t0, t0 + 2 * DAY)
    eng.set_phase_timing(1)
    try:
        lean = eng.expand(sp, ny, t0, t0 + 2 * DAY)
        kt = eng.kernel_times()
    finally:
        eng.set_phase_timing(2)
    assert np.array_equal(full[0], lean[0]) and np.array_equal(full[1], lean[1])
    assert kt[3] > 0 and kt[0] == kt[1] == kt[2] == kt[4] == kt[5] == -1
    with pytest.raises(_lib.CgError):
        eng.set_phase_timing(3)


def test_output_growth_and_reuse():
    """A fresh context: first call (no output buffer: separate slice map),
    a larger call (E beyond the capacity: the scan's slice map is discarded,
    buffers grow, the write phase reruns), then smaller calls that reuse the
    capacity (slice map built by the scan) -- all bit-exact."""
    from cronsun_amd.engine import Engine
    eng = Engine(0)
    rng = np.random.default_rng(21)
    small = [cron.Parse(random_spec(rng)) for _ in range(300)]
    big = small + [cron.Parse("*/2 * * * * *")] * 40 + [cron.Parse(random_spec(rng)) for _ in range(700)]
    t0 = synth.T0_2026
    for scheds, t1 in ((small, t0 + DAY), (big, t0 + 2 * DAY), (small, t0 + DAY), (big, t0 + DAY)):
        check_same(eng, scheds, "UTC", t0, t1)


@pytest.mark.parametrize("t0", [1772910000, 1793469600, 1773792000], ids=["ny-spring", "ny-fall", "ny-spring+10d"])
def test_config2_scale_dst_day(eng, t0):
    """Config 2 at full size in America/New_York over the 24 h centred on the
    2026 spring-forward / fall-back (clean transitions: the closed form cut at
    the transition, the fall-back overlap's repeated hour), and over a day ten
    days after the spring-forward (a walk from T0 could reset back across it),
    bit-exact on a seeded sample that includes every every-second rule."""
    n = 1_000_000
    specs = synth.spec_mix(n, seed=0x5EED)
    arr, status = cron.parse_batch(specs)
    assert (status == 0).all()
    sp = eng.upload_c(arr, n)
    t1 = t0 + DAY
    E = eng.expand_device(sp, product_zone("America/New_York"), t0, t1)
    off = np.empty(n + 1, dtype=np.int64)
    from cronsun_amd._lib import check, lib
    check(lib().cg_result_copy_offsets(eng._h, off.ctypes.data))
    assert off[0] == 0 and off[-1] == E and (np.diff(off) >= 0).all()
    times = eng.copy_times(0, E)
    assert ((times > t0) & (times <= t1)).all()
    steps = np.nonzero(np.diff(times) <= 0)[0] + 1
    assert np.isin(steps, off[1:-1]).all()
    rng = np.random.default_rng(t0 & 0xFFFF)
    heavy = [i for i in range(n) if specs[i] == "* * * * * *"][:200]
    idx = np.unique(np.concatenate([rng.choice(n, 3000, replace=False), np.array(heavy, dtype=np.int64)]))
    sample = [cron.Parse(specs[i]) for i in idx]
    eo, et = oracle_csr(sample, "America/New_York", t0, t1, [specs[i] for i in idx])
    for k, i in enumerate(idx):
        assert np.array_equal(times[off[i]:off[i + 1]], et[eo[k]:eo[k + 1]]), specs[i]
    sp.free()


def test_async_pipeline(eng):
    """cg_expand_device_async / cg_expand_wait: a scheduler's consecutive
    windows (T0 moving every call, America/New_York over the 2026
    spring-forward) pipelined; the last call's result equals the synchronous
    expansion of its window and the oracle; an oversized result is reported
    as CG_ECAPACITY, a never-ending reference loop as CG_ERANGE (Pacific/Apia
    over the skipped 2011-12-30), each at the wait."""
    from cronsun_amd.engine import Engine
    specs = synth.spec_mix(20_000, seed=11)
    arr, status = cron.parse_batch(specs)
    assert (status == 0).all()
    e2 = Engine(0)
    sp = e2.upload_c(arr, len(specs))
    ny = product_zone("America/New_York")
    t0 = 1772953200 - 30 * 3600
    e2.expand_device(sp, ny, t0, t0 + 3 * DAY)  # sizes the output for the windows below
    wins = [(t0 + 6 * 3600 * i, t0 + 6 * 3600 * i + DAY) for i in range(7)]
    for a, b in wins:
        e2.expand_async(sp, ny, a, b)
    E = e2.expand_wait()
    off = np.empty(len(specs) + 1, dtype=np.int64)
    from cronsun_amd._lib import check, lib
    check(lib().cg_result_copy_offsets(e2._h, off.ctypes.data))
    times = e2.copy_times(0, E)
    a, b = wins[-1]
    E_sync = e2.expand_device(sp, ny, a, b)
    off_s = np.empty_like(off)
    check(lib().cg_result_copy_offsets(e2._h, off_s.ctypes.data))
    assert E == E_sync and np.array_equal(off, off_s)
    assert np.array_equal(times, e2.copy_times(0, E_sync))
    idx = np.arange(0, len(specs), 7)
    eo, et = oracle_csr([cron.Parse(specs[i]) for i in idx], "America/New_York", a, b, [specs[i] for i in idx])
    for k, i in enumerate(idx):
        assert np.array_equal(times[off[i]:off[i + 1]], et[eo[k]:eo[k + 1]]), specs[i]
    # capacity: a window far larger than the output sized above
    e2.expand_async(sp, ny, t0, t0 + 30 * DAY)
    with pytest.raises(_lib.CgError) as err:
        e2.expand_wait()
    assert err.value.code == _lib.CG_ECAPACITY
    sp.free()
    # a rule whose reference loop never ends, among ordinary ones
    stuck = [cron.Parse(s) for s in ["0 0 12 * * *", "0 0 9 * * Sat", "@daily"]]
    sp2 = e2.upload(stuck)
    apia = product_zone("Pacific/Apia")
    e2.expand_device(sp2, apia, 1325030400 - 10 * DAY, 1325030400 - 5 * DAY)
    e2.expand_async(sp2, apia, 1325030400 - 10 * DAY, 1325030400 - 5 * DAY)
    e2.expand_async(sp2, apia, 1325030400, 1325030400 + 5 * DAY)
    with pytest.raises(_lib.CgError) as err:
        e2.expand_wait()
    assert err.value.code == _lib.CG_ERANGE and "rule 1:" in err.value.msg
    e2.close()


@pytest.mark.parametrize("zone", ["America/New_York", "America/Havana", "Australia/Lord_Howe",
                                  "Pacific/Chatham", "Pacific/Apia", "Europe/Dublin"])
def test_starts_near_transitions(eng, zone):
    """T0 just before, on, inside the overlap of, and hours / a day after zone
    transitions of 2011-2027 (Pacific/Apia's skipped 2011-12-30 included):
    the narrowed WALK windows, Next(T0) by the exact walk after a recent
    transition, and the last Next walked to its end before a skipped day --
    the kernels against the oracle (the host check in tests/native covers
    more starts)."""
    from test_zone import _table
    z = product_zone(zone)
    when, off = _table(z, 1293840000, 1830297600)
    idx = list(range(1, len(when), max(1, (len(when) - 1) // 3)))[:3]
    big = 1 + int(np.argmax(np.abs(np.diff(off))))
    if big not in idx:
        idx.append(big)
    rng = np.random.default_rng(zlib.crc32(("near" + zone).encode()))
    specs = [random_spec(rng) for _ in range(150)] + ["0 30 2 * * *", "0 0 0 * * *", "0 0 9 * * Sat",
                                                      "0 0 1 * * *", "0 */15 * * * *"]
    scheds = [cron.Parse(s) for s in specs]
    for i in idx:
        tau = int(when[i])
        for o in (-3600, -1, 0, 1, 3599, 3601, 18001, 90000):
            check_same(eng, scheds, zone, tau + o, tau + o + 30 * 3600, specs)


_SHORT = {}


def _short_window_rules(n):
    """config-2 specs and their oracle parse (cached across the parametrized cases)"""
    if n not in _SHORT:
        specs = synth.spec_mix(n, seed=0x5EED)
        _SHORT[n] = specs, O.sched_array(oracle_parse_all(specs))
    return _SHORT[n]


@pytest.mark.parametrize("width", [60, 3600])
def test_short_windows_after_a_day(eng, width):
    """Short windows (the writer's cost-space slices, cg_kernels.h u_mode) of
    300k config-2 rules, expanded right after a 24-h call grew the output (so the
    capacity is far above the window's events): the whole rule-major CSR
    bit-exact against the oracle, at a window start on and off a minute."""
    n = 300_000
    specs, oarr = _short_window_rules(n)
    arr, status = cron.parse_batch(specs)
    assert (status == 0).all()
    sp = eng.upload_c(arr, n)
    eng.expand_device(sp, None, synth.T0_2026, synth.T0_2026 + DAY)
    from cronsun_amd._lib import check, lib
    for t0 in (synth.T0_2026 + 7 * 3600, synth.T0_2026 + 7 * 3600 + 37):
        t1 = t0 + width
        E = eng.expand_device(sp, None, t0, t1)
        off = np.empty(n + 1, dtype=np.int64)
        check(lib().cg_result_copy_offsets(eng._h, off.ctypes.data))
        times = eng.copy_times(0, E)
        eo, et = O.expand_batch(oarr, t0, t1, oracle_zone("UTC"), threads=8)
        assert np.array_equal(off, eo), (width, t0)
        assert np.array_equal(times, et), (width, t0)


def test_async_result_hygiene():
    """cg_expand_wait with nothing pending sets n_events = 0; the result
    accessors refuse while asynchronous calls are pending; a synchronous call
    made while a failing asynchronous call is pending discards that call's
    error (the next wait reports only its own calls)."""
    from cronsun_amd.engine import Engine
    from cronsun_amd._lib import check, lib
    e2 = Engine(0)
    specs = synth.spec_mix(5_000, seed=13)
    arr, status = cron.parse_batch(specs)
    sp = e2.upload_c(arr, len(specs))
    t0 = synth.T0_2026
    E = e2.expand_device(sp, None, t0, t0 + DAY)
    assert e2.expand_wait() == 0
    e2.expand_async(sp, None, t0, t0 + DAY)
    off = np.empty(len(specs) + 1, dtype=np.int64)
    with pytest.raises(_lib.CgError) as err:
        check(lib().cg_result_copy_offsets(e2._h, off.ctypes.data))
    assert err.value.code == _lib.CG_EINVAL
    assert e2.expand_wait() == E
    check(lib().cg_result_copy_offsets(e2._h, off.ctypes.data))
    assert off[-1] == E
    e2.expand_async(sp, None, t0, t0 + 30 * DAY)  # exceeds the capacity: CG_ECAPACITY at a wait
    E2 = e2.expand_device(sp, None, t0, t0 + 3600)  # drains and discards it
    e2.expand_async(sp, None, t0, t0 + 3600)
    assert e2.expand_wait() == E2
    sp.free()
    e2.close()
