"""The C-ABI from plain C (tests/native/abi_c.c, gcc -std=c11 -pedantic
-Werror against include/cronsun_gpu.h), in the call order of the cgo stub
node/cron/gpu/gpu.go (the boundary of node/cron/cron.go:36-40 and
parser.go:181-183).  CPU: the header compiles as C11, the program links and
runs its host-side calls (parser, zones, jobset), and cg_init reports
CG_ENODEV.  GPU: every result it prints is compared with the oracle."""
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O
from common import ZONEINFO, oracle_zone

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "abi_c.c")
BIN = os.path.join(ROOT, "tests", "native", "abi_c")
LIBDIR = os.path.join(ROOT, "cronsun_amd")
SPECS = ["0 */5 * * * *", "0 30 9 * * 1-5", "0 0 12 1,15 * Mon", "@daily", "@every 90s", "*/10 * * * * *",
         "0 0 0 30 Feb ?", "15/35 20-35/15 1/2 */2 * *", "0 30 2 * * *", "0 0 0 29 Feb ?", "@hourly",
         "59 59 23 * * Sun"]


@pytest.fixture(scope="module")
def abi_c():
    lib = os.path.join(LIBDIR, "libcronsun_gpu.so")
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(os.path.getmtime(SRC), os.path.getmtime(lib)):
        subprocess.check_call(["gcc", "-std=c11", "-pedantic", "-Wall", "-Wextra", "-Werror", "-O2", "-o", BIN,
                               SRC, "-L" + LIBDIR, "-lcronsun_gpu", "-Wl,-rpath," + LIBDIR])
    return BIN


def _run(abi_c, *args, timeout=120):
    out = subprocess.run([abi_c, ZONEINFO] + list(args), capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    lines = {}
    for ln in out.stdout.splitlines():
        k, _, rest = ln.partition(" ")
        lines.setdefault(k, []).append(rest)
    return lines


def test_header_is_c11_and_host_calls_run(abi_c):
    from cronsun_amd import engine
    lines = _run(abi_c, "check")
    assert lines["P"][0].startswith("parse_error ")
    assert lines["P"][0][len("parse_error "):] == O.parse("* * *")[1]  # Go's message (parser.go:95-100)
    assert lines["Z"] == ["offset_after_spring_forward -14400"]
    assert lines["J"] == ["rules 12 nodes 5 groups 2 jobs 12"]
    if engine.device_count() == 0:
        assert "NODEV" in lines


def _oracle_scheds():
    return [O.parse(s)[0] for s in SPECS]


@pytest.mark.gpu
def test_call_sequence_matches_oracle(abi_c):
    lines = _run(abi_c, "check")
    assert "OK" in lines
    ny = oracle_zone("America/New_York")
    sch = _oracle_scheds()
    tin = [1772953200 - 3600 + 977 * i for i in range(len(SPECS))]
    assert [int(x) for x in lines["N"][0].split()] == [O.sched_next(s, t, ny) for s, t in zip(sch, tin)]
    t0 = 1772953200 - 12 * 3600
    t1 = t0 + 2 * 86400
    eo, et = O.expand_batch(O.sched_array(sch), t0, t1, ny)
    e = [int(x) for x in lines["E"][0].split()]
    assert e[0] == eo[-1] and e[1:] == eo.tolist()
    assert [int(x) for x in lines["T"][0].split()] == et.tolist()
    # per node: the C program's jobset, restated as integer arrays for the oracle
    groups = {"g1": ["n1", "n2", "n3"], "g2": ["n3", "n4"]}
    nodes = []
    for g in ("g1", "g2"):
        for n in groups[g]:
            if n not in nodes:
                nodes.append(n)
    nodes.append("n5")
    R = len(SPECS)
    from cronsun_amd.engine import RulesIn
    gl = [[nodes.index(n) for n in groups[g]] for g in ("g1", "g2")]
    rin = RulesIn(len(nodes), 2, R, R,
                  group_off=np.cumsum([0] + [len(x) for x in gl]), group_nodes=sum(gl, []),
                  group_exists=[1, 1], rule_job=np.arange(R),
                  nid_off=np.cumsum([0] + [int(i % 3 == 0) for i in range(R)]),
                  nids=[nodes.index("n5")] * sum(int(i % 3 == 0) for i in range(R)),
                  gid_off=np.arange(R + 1), gids=[0 if i % 2 else 1 for i in range(R)],
                  ex_off=np.cumsum([0] + [int(i % 4 == 0) for i in range(R)]),
                  ex=[nodes.index("n3")] * sum(int(i % 4 == 0) for i in range(R)),
                  job_pause=[int(i == 7) for i in range(R)])
    roff, rules = O.node_rules(rin, 0, np.arange(len(nodes)))
    got = {ln.split(" ", 1)[0]: ln.split(" ")[1:] for ln in lines["L"]}
    got_o = {ln.split(" ", 1)[0]: ln.split(" ")[1:] for ln in lines["O"]}
    got_q = {ln.split(" ", 1)[0]: ln.split(" ")[1:] for ln in lines["Q"]}  # cg_set_node_order(TIME)
    for k, name in enumerate(nodes):
        exp_t, exp_r = O.node_list(eo, et, rules[roff[k]:roff[k + 1]])
        want = [f"{r}:{t}" for r, t in zip(exp_r.tolist(), exp_t.tolist())]
        assert [x for x in got.get(name, []) if x] == want, name
        o = np.lexsort((exp_r, exp_t))  # byTime, equal times in rule order
        want_o = [f"{r}:{t}" for r, t in zip(exp_r[o].tolist(), exp_t[o].tolist())]
        assert [x for x in got_o.get(name, []) if x] == want_o, name
        assert [x for x in got_q.get(name, []) if x] == want_o, name
    kind = [i % 3 for i in range(R)]
    avg = [1000 * i - 2500 for i in range(R)]
    assert [int(x) for x in lines["K"][0].split()] == [
        O.lock_ttl(s, t, ny, k, a, 300) for s, t, k, a in zip(sch, tin, kind, avg)]
    # the dispatcher: three wakes, slot 2 replaced by @every 90s and slot 5 removed after the first
    oc = O.OracleCron(sch, ny)
    oc.start(t0)
    for w, ln in enumerate(lines["W"]):
        f = [int(x) for x in ln.split()]
        eff = oc.effective()
        assert f[0] == eff, w
        assert f[1:] == oc.fire(eff, eff), w
        if w == 0:
            oc.set(2, sch[4], eff)
            oc.remove(5)


@pytest.mark.gpu
def test_c_consumer_expansion_rate(abi_c, tmp_path):
    """BASELINE config 2 (1M mixed rules x 24 h, UTC) driven from C with no
    PyTorch in the process: the per-step time a cgo caller sees."""
    from cronsun_amd import synth
    p = os.path.join(str(tmp_path), "specs.txt")
    with open(p, "w") as f:
        f.write("\n".join(synth.spec_mix(1_000_000, seed=0x5EED)))
    lines = _run(abi_c, "bench", p, timeout=300)
    b = lines["B"][0].split()
    rec = dict(zip(b[0::2], b[1::2]))
    print("C consumer:", rec)
    if os.environ.get("CG_TEST_RECORD_DIR"):  # tools/gpu_check.sh keeps the record
        import json
        with open(os.path.join(os.environ["CG_TEST_RECORD_DIR"], "abi_c_bench.json"), "w") as f:
            json.dump(rec, f)
    assert int(rec["rules"]) == 1_000_000 and int(rec["events"]) == 674766895
