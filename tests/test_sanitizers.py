"""The library's host parsers under AddressSanitizer + UBSan (CPU only).

Everything that reaches libcronsun_gpu.so from outside is parsed on the host:
etcd JSON values of jobs and groups (cg_ingest.cpp restating Go 1.8
encoding/json for job.go:38-84 / group.go:17-22, then Job.Valid and the
interning in cg_jobset.cpp), cron spec strings (cg_parse.cpp, parser.go:78-377),
durations of "@every" and TZif zone files (cg_zone.cpp: LoadLocationFromTZData
+ the plan builder).  tests/native/fuzz_host.cpp drives those sources, built
with -fsanitize=address,undefined and no recovery, over: the seeded JSON
mutation corpus of test_ingest.py (3000 job documents), garbage and valid
specs, and every committed TZif file plus truncations and byte-level
corruptions of them.  Any out-of-bounds access, use-after-free, leak or
undefined behaviour aborts the driver."""
import os
import struct
import subprocess

import numpy as np
import pytest

from common import ZONEINFO, garbage_spec, random_spec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cronsun_amd", "csrc")
SRC = os.path.join(ROOT, "tests", "native", "fuzz_host.cpp")
BIN = os.path.join(ROOT, "tests", "native", "fuzz_host_asan")
HOST_SRCS = [os.path.join(CSRC, f) for f in ("cg_parse.cpp", "cg_zone.cpp", "cg_ingest.cpp", "cg_jobset.cpp")]
ZONES = ["UTC", "America/New_York", "Europe/London", "Australia/Lord_Howe", "America/Havana",
         "Pacific/Apia", "Africa/Casablanca", "Asia/Kathmandu", "Pacific/Chatham", "Europe/Dublin"]


@pytest.fixture(scope="module")
def fuzz_bin():
    deps = [SRC] + HOST_SRCS + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    if not os.path.exists(BIN) or any(os.path.getmtime(BIN) < os.path.getmtime(d) for d in deps):
        subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
                               "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                               "-o", BIN, SRC] + HOST_SRCS + ["-lpthread"])
    return BIN


def _write(path, records):
    with open(path, "wb") as f:
        for kind, b in records:
            f.write(struct.pack("<II", kind, len(b)))
            f.write(b)


def _run(fuzz_bin, tmp_path, records):
    path = os.path.join(tmp_path, "in.bin")
    _write(path, records)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    out = subprocess.run([fuzz_bin, path], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-6000:]
    return out.stdout


def test_json_ingestion_under_asan_ubsan(fuzz_bin, tmp_path):
    from test_ingest import _random_doc, J
    rng = np.random.default_rng(20261016)
    jobs = [_random_doc(rng) for _ in range(3000)]
    groups = [J({"id": f"g{i % 40}", "nids": [f"n{int(x)}" for x in rng.integers(0, 40, 3)]}).encode()
              for i in range(60)]
    # hostile shapes beyond the mutation corpus: deep nesting, huge numbers,
    # escapes, invalid UTF-8, NUL bytes in IDs, truncations of every length
    nasty = [b"[" * 5000 + b"]" * 5000, b'{"id":' + b"9" * 400 + b"}", b'{"id":"\\ud800\\udc00x"}',
             b'{"id":"\\u00"}', b'{"id":"a\x00b","rules":[]}', b'{"id":"\xff\xfe","rules":[{"timer":"@daily"}]}',
             b'{"rules":[null,{"id":null,"timer":null}]}', b'{"id":"x","rules":[{"timer":"' + b"*" * 10000 + b'"}]}',
             b"", b"{", b'{"id":"x",}', b"null", b'"str"', b"1e999", b'{"kind":1e400}',
             b'{"avg_time":-9223372036854775809}', b'{"parallels":18446744073709551616}']
    doc = jobs[7]
    nasty += [doc[:i] for i in range(len(doc))]
    gnasty = [b'{"id":"g","nids":[' + b'"n",' * 3000 + b'"n"]}', b'{"id":"g2","nids":null}',
              b'{"id":"g3","nids":"n"}', b'{"ID":"g4","NIDS":["a"]}']
    out = _run(fuzz_bin, str(tmp_path), [(0, g) for g in groups + gnasty] + [(1, d) for d in jobs + nasty])
    assert "accepted" in out


def test_spec_and_duration_parsers_under_asan_ubsan(fuzz_bin, tmp_path):
    rng = np.random.default_rng(99)
    specs = [garbage_spec(rng).encode() for _ in range(4000)] + \
            [random_spec(rng).encode() for _ in range(2000)]
    specs += [b"", b" ", b"@", b"@every", b"@every ", b"@every -", b"* * * * * * * *", b"\x00",
              b"*/" + b"9" * 40 + b" * * * * *", b"1-" + b"9" * 30 + b" * * * * *",
              b"@every " + b"9" * 40 + b"h", b"\xff\xfe * * * * *"]
    durs = [b"1h", b"1.5h", b".5s", b"-1s", b"9223372036854775807ns", b"9223372036854775808ns",
            b"1" + b"0" * 40 + b"s", b"3\xc2\xb5s", b"1us2ms", b"", b"h", b"1", b"1.", b"+.0s", b"-0"]
    fields = [b"*", b"?", b"*/0", b"5-3", b"1-" + b"9" * 25, b"jan-dec/2", b"mon-sun", b",,", b"-",
              b"*/" + b"4" * 30, b"x-y", b"1,2,,3", b"\x00"]
    out = _run(fuzz_bin, str(tmp_path), [(2, s) for s in specs] + [(4, d) for d in durs] +
               [(5, f) for f in fields])
    assert "spec-parses=" in out


def test_tzif_reader_under_asan_ubsan(fuzz_bin, tmp_path):
    rng = np.random.default_rng(7)
    blobs = []
    for z in ZONES:
        with open(os.path.join(ZONEINFO, z), "rb") as f:
            data = f.read()
        blobs.append(data)
        blobs += [data[:i] for i in range(0, len(data), max(1, len(data) // 97))]  # truncations
        for _ in range(60):  # byte-level corruptions, incl. the counts in the header
            b = bytearray(data)
            for _ in range(int(rng.integers(1, 6))):
                i = int(rng.integers(0, len(b)))
                b[i] = int(rng.integers(0, 256))
            blobs.append(bytes(b))
        hdr = bytearray(data)
        for off in range(20, 44, 4):  # every header count set to a huge value
            h = bytearray(hdr)
            h[off:off + 4] = b"\x7f\xff\xff\xff"
            blobs.append(bytes(h))
        blobs.append(data[:-1] + b"<+99>-99<-99>,M13.9.9/999,J999")  # broken footer
    out = _run(fuzz_bin, str(tmp_path), [(3, b) for b in blobs])
    assert "tzif=" in out
