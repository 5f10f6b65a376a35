"""The expansion algorithm the kernels run (cg_expand.h: count_rule with the
closed-form first fire, closed-form iteration, WALK re-walk), compiled for the
host and checked fire-by-fire against the oracle's literal Next loop
(t = Next(t) until > T1) on random specs over zones with DST, midnight and
30/45-minute transitions (tests/native/expand_host.cpp).  CPU only: the GPU
tests check the kernels themselves."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "expand_host.cpp")
BIN = os.path.join(ROOT, "tests", "native", "expand_host")


@pytest.fixture(scope="module")
def expand_host():
    import oracle_lib as O
    O.lib()  # builds oracle/liboracle.so if needed
    srcs = [SRC, os.path.join(ROOT, "cronsun_amd", "csrc", "cg_zone.cpp")]
    if not os.path.exists(BIN) or any(os.path.getmtime(BIN) < os.path.getmtime(s) for s in srcs + [
            os.path.join(ROOT, "cronsun_amd", "csrc", "cg_expand.h"),
            os.path.join(ROOT, "cronsun_amd", "csrc", "cg_time.h")]):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", BIN] + srcs +
                              ["-L" + os.path.join(ROOT, "oracle"), "-loracle",
                               "-Wl,-rpath," + os.path.join(ROOT, "oracle")])
    return BIN


@pytest.mark.parametrize("zone", ["UTC", "America/New_York", "Europe/London", "Australia/Sydney",
                                  "America/Havana", "Australia/Lord_Howe", "Asia/Kathmandu",
                                  "Pacific/Chatham", "America/St_Johns", "Africa/Casablanca",
                                  "Pacific/Apia"])
def test_host_algorithm_matches_oracle(expand_host, zone):
    out = subprocess.run([expand_host, zone, "300", "11"], cwd=ROOT, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert " 0 mismatches" in out.stdout


@pytest.mark.parametrize("zone", ["UTC", "America/New_York", "Australia/Lord_Howe", "Africa/Casablanca"])
def test_host_algorithm_long_horizons(expand_host, zone):
    """Multi-year horizons (3 years from 2026; 2095-2106, where Feb 29 skips
    2100 and Next's five-year limit returns the zero time, spec.go:70-76)."""
    out = subprocess.run([expand_host, zone, "60", "5", "long"], cwd=ROOT, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert " 0 mismatches" in out.stdout


@pytest.mark.parametrize("zone", ["America/New_York", "Europe/Dublin", "America/Havana", "Australia/Lord_Howe",
                                  "Pacific/Chatham", "Pacific/Apia", "Africa/Casablanca", "America/Sao_Paulo"])
def test_host_algorithm_near_transitions(expand_host, zone):
    """T0 at 18 offsets around six transitions of 2011-2027 (just before, on,
    inside a backward transition's overlap, hours and days after; Pacific/Apia's
    skipped 2011-12-30 included): narrow WALK windows, Next(T0) by the exact
    walk after a recent transition, and the reference's last Next past T1
    walked to its end where a skipped day could stall it."""
    out = subprocess.run([expand_host, zone, "150", "13", "near"], cwd=ROOT, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert " 0 mismatches" in out.stdout


@pytest.mark.parametrize("zone", ["America/New_York", "Europe/London", "Australia/Sydney", "America/St_Johns",
                                  "Africa/Casablanca"])
def test_host_algorithm_clean_transitions(expand_host, zone):
    """Every clean transition of 2011-2027 (cg_zone.cpp clean_transition: a
    one-hour shift at a local hour start away from midnight -- the plan cuts
    the closed form there, with no WALK window and no exact walk from T0):
    T0 at 16 offsets around it (30-h horizons) and on days 1-39 after it
    (24-h horizons).  Every such plan must run without an exact walk."""
    out = subprocess.run([expand_host, zone, "60", "17", "clean"], cwd=ROOT, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert " 0 mismatches" in out.stdout
    line = [l for l in out.stdout.splitlines() if "planned without any exact walk" in l][0]
    n_clean, n_all = int(line.split(": ")[1].split()[0]), int(line.split(" of ")[1].split()[0])
    assert n_all > 100 and n_clean == n_all, line
