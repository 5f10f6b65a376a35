"""Shared helpers for the parity tests."""
import ctypes as C
import os

import numpy as np

import oracle_lib as O

ZONES = ["UTC", "America/New_York", "Europe/London", "Australia/Sydney", "America/Havana",
         "Australia/Lord_Howe", "Asia/Kathmandu", "Asia/Kolkata", "America/Sao_Paulo",
         "Pacific/Chatham", "Europe/Dublin", "America/St_Johns", "Africa/Casablanca",
         "Pacific/Apia", "fixed:19800", "fixed:-34200"]

ZONEINFO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "zoneinfo")


def product_zone(name):
    from cronsun_amd import cron
    if name == "UTC":
        return cron.UTC()
    if name.startswith("fixed:"):
        return cron.FixedZone(name, int(name.split(":")[1]))
    with open(os.path.join(ZONEINFO, name), "rb") as f:
        return cron.LoadLocationFromTZData(name, f.read())


_oracle_locs = {}


def oracle_zone(name):
    if name not in _oracle_locs:
        _oracle_locs[name] = O.Loc(name)
    return _oracle_locs[name]


FIELD_ATOMS = {
    0: ["*", "?", "0", "5", "59", "*/7", "0/15", "15/35", "10-20", "10-40/3", "1,2,3", "7,30,45",
        "*/1", "58-59", "0-59/59", "3-3"],
    1: ["*", "0", "30", "*/5", "0/15", "20-35/15", "1,31,59", "5-7/2", "*/59", "10-12"],
    2: ["*", "0", "9", "23", "*/2", "1/2", "9-17", "22,23,0", "0-23/5", "2", "1", "3"],
    3: ["*", "?", "1", "15", "31", "29", "30", "1,15", "*/2", "9-20", "*/10", "28-31", "5/7"],
    4: ["*", "?", "1", "2", "Feb", "Jan,Jul", "Apr-Oct", "*/3", "Mar", "Nov", "Dec", "jun-AUG", "2-2"],
    5: ["*", "?", "0", "1-5", "Mon", "Sun", "mon/2", "Sat,Sun", "*/2", "3", "fri-sat", "0-6/3"],
}


def random_spec(rng):
    """A random six-field spec over the full grammar (mostly valid)."""
    r = rng.random()
    if r < 0.05:
        return ["@yearly", "@annually", "@monthly", "@weekly", "@daily", "@midnight",
                "@hourly"][rng.integers(0, 7)]
    if r < 0.12:
        return f"@every {rng.integers(1, 7200)}s"
    fields = [FIELD_ATOMS[i][rng.integers(0, len(FIELD_ATOMS[i]))] for i in range(6)]
    if rng.random() < 0.2:
        fields = fields[:5]
    return " ".join(fields)


GARBAGE_ATOMS = ["", "*", "-", "/", ",", "5--5", "*//2", "*/-1", "x", "Jan", "mon", "60", "24",
                 "32", "13", "7", "0", "+5", "05", "1-", "-1", "5-3", "*/0", "*-5", "?/2",
                 "99999999999999999999", "1,,2", "@", "\t", "jan-x", "3/", "/3"]


def garbage_spec(rng):
    n = int(rng.integers(0, 8))
    parts = []
    for _ in range(n):
        a = GARBAGE_ATOMS[rng.integers(0, len(GARBAGE_ATOMS))]
        if rng.random() < 0.3:
            a = a + GARBAGE_ATOMS[rng.integers(0, len(GARBAGE_ATOMS))]
        parts.append(a)
    sep = [" ", "  ", "\t", " \n "][rng.integers(0, 4)]
    s = sep.join(parts)
    if rng.random() < 0.1:
        s = "@every " + ["5m", "1h30m", "Xm", "1.5h", ".5s", "5", "-1s", "0", "1us", "3µs"][
            rng.integers(0, 10)]
    return s


def to_oracle_sched(cs):
    """cg_schedule (product) -> OrSched (oracle)"""
    s = O.OrSched()
    s.kind = cs.kind
    s.delay_ns = cs.delay_ns
    s.spec.second, s.spec.minute, s.spec.hour = cs.second, cs.minute, cs.hour
    s.spec.dom, s.spec.month, s.spec.dow = cs.dom, cs.month, cs.dow
    return s


def oracle_parse_all(specs):
    out = []
    for sp in specs:
        s, err = O.parse(sp)
        assert err is None, (sp, err)
        out.append(s)
    return out
