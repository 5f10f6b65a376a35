"""Pin the CPU oracle against every known-answer case the reference's own
tests hold for this path (tests/golden/kats.json, transcribed from
node/cron/spec_test.go, constantdelay_test.go, parser_test.go)."""
import ctypes as C
import json
import os

import pytest

import oracle_lib as O

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kats.json")))
_LOCS = {}


def loc(name):
    if name not in _LOCS:
        _LOCS[name] = O.Loc(name)
    return _LOCS[name]


def test_kat_row_counts():
    # 74 Next-style rows + 4 errors, 14 constant-delay, 45 parser rows
    assert len(KATS["activation"]) + len(KATS["next"]) + len(KATS["next_tz"]) == 74
    assert len(KATS["errors"]) == 4
    assert len(KATS["constant_delay"]) == 14
    parser = sum(len(KATS[k]) for k in ("range", "field", "all", "bits", "parse", "parse_standard"))
    assert parser == 45


@pytest.mark.parametrize("row", KATS["activation"], ids=lambda r: r["ref"])
def test_activation(row):
    s, err = O.parse(row["spec"])
    assert err is None, err
    actual = O.sched_next(s, row["time"] - 1, loc(row["zone"]))
    assert (actual == row["time"]) == row["expected"]


@pytest.mark.parametrize("row", KATS["next"] + KATS["next_tz"], ids=lambda r: r["ref"])
def test_next(row):
    s, err = O.parse(row["spec"])
    assert err is None, err
    assert O.sched_next(s, row["time"], loc(row["zone"])) == row["expected"]


@pytest.mark.parametrize("row", KATS["errors"], ids=lambda r: r["ref"])
def test_errors(row):
    s, err = O.parse(row["spec"])
    assert s is None and err


@pytest.mark.parametrize("row", KATS["constant_delay"], ids=lambda r: r["ref"])
def test_constant_delay(row):
    L = O.lib()
    d = L.or_every(row["delay_ns"])
    assert L.or_const_next(d, row["time"], row["nsec"]) == row["expected"]


def _range(fn, row):
    bits = C.c_uint64()
    err = C.create_string_buffer(512)
    b = row["expr"].encode()
    rc = fn(b, len(b), row["min"], row["max"], C.byref(bits), err, 512)
    return rc, bits.value, err.value.decode()


@pytest.mark.parametrize("row", KATS["range"], ids=lambda r: r["ref"])
def test_range(row):
    rc, bits, err = _range(O.lib().or_get_range, row)
    if row["err"]:
        assert rc != 0 and row["err"] in err
    else:
        assert rc == 0, err
    assert bits == int(row["expected"])


@pytest.mark.parametrize("row", KATS["field"], ids=lambda r: r["ref"])
def test_field(row):
    rc, bits, _ = _range(O.lib().or_get_field, row)
    assert bits == int(row["expected"])


@pytest.mark.parametrize("row", KATS["all"], ids=lambda r: r["ref"])
def test_all(row):
    assert (O.lib().or_get_bits(row["min"], row["max"], 1) | (1 << 63)) == int(row["expected"])


@pytest.mark.parametrize("row", KATS["bits"], ids=lambda r: r["ref"])
def test_bits(row):
    assert O.lib().or_get_bits(row["min"], row["max"], row["step"]) == int(row["expected"])


def _check_parse(row, options):
    s, err = O.parse(row["expr"], options)
    if row["err"]:
        assert s is None and row["err"] in err
        return
    assert err is None, err
    exp = row["expected"]
    if exp["kind"] == "every":
        assert s.kind == 1 and s.delay_ns == exp["delay_ns"]
    else:
        assert s.kind == 0
        for f in ("second", "minute", "hour", "dom", "month", "dow"):
            assert getattr(s.spec, f) == int(exp[f]), f


@pytest.mark.parametrize("row", KATS["parse"], ids=lambda r: r["ref"])
def test_parse(row):
    _check_parse(row, O.OPT_DEFAULT)


@pytest.mark.parametrize("row", KATS["parse_standard"], ids=lambda r: r["ref"])
def test_parse_standard(row):
    _check_parse(row, O.OPT_STANDARD)
