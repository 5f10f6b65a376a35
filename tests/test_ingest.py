"""Bulk ingestion of cronsun's etcd values (cg_jobset_ingest_*, C++) against
the oracle's restatement of Go 1.8 encoding/json + GetJobs/GetGroups
(oracle/go_json.py): statuses, and for every ingested job its ID, Pause,
Kind, AvgTime, Parallels (after alone()), rules (ID, gids, nids,
exclude_nids) and parsed schedules.  Hand-written cases pin the
encoding/json rules that matter (key folding, duplicates, slice element
reuse, null, type errors, escapes); seeded mutations of valid documents cover
the rest.  CPU only (host code)."""
import ctypes as C
import json
import os
import sys

import numpy as np
import pytest

import oracle_lib as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import go_json as G  # noqa: E402


def _oparse(timer):
    s = O.OrSched()
    err = C.create_string_buffer(512)
    rc = O.lib().or_parse(O.OPT_DEFAULT, timer, len(timer), C.byref(s), err, 512)
    return s if rc == 0 else None


def _product(job_docs, group_docs=()):
    from cronsun_amd.ingest import EtcdJobSet
    return EtcdJobSet(job_docs, group_docs, threads=4)


def _compare(job_docs, group_docs=()):
    js = _product(job_docs, group_docs)
    ost, ojobs = G.ingest_jobs(job_docs, _oparse)
    gst, ogroups = G.ingest_groups(group_docs)
    assert list(js.job_status) == ost
    assert list(js.group_status) == gst
    assert js.n_jobs == len(ojobs)
    rin = js.rules_in()
    kind, avg, par = js.job_meta()
    scheds = js.schedules_c() if js.n_rules else []
    r = 0
    for jx, (_, oj) in enumerate(ojobs):
        assert js.job_id(jx) == oj["id"]
        assert bool(rin.job_pause[jx]) == oj["pause"]
        assert (int(kind[jx]), int(avg[jx]), int(par[jx])) == (oj["kind"], oj["avg_time"], oj["parallels"])
        for orule, osch in zip(oj["rules"].items(), oj["schedules"]):
            assert int(rin.rule_job[r]) == jx
            assert js.rule_id(r) == orule["id"]
            nid = [js.node_id(int(x)).encode() if js.node_id(int(x)) is not None else None
                   for x in rin.nids[rin.nid_off[r]:rin.nid_off[r + 1]]]
            assert [lib_node(js, int(x)) for x in rin.nids[rin.nid_off[r]:rin.nid_off[r + 1]]] == \
                orule["nids"].items(), nid
            assert [lib_node(js, int(x)) for x in rin.ex[rin.ex_off[r]:rin.ex_off[r + 1]]] == \
                orule["exclude_nids"].items()
            assert [js.group_id(int(x)) for x in rin.gids[rin.gid_off[r]:rin.gid_off[r + 1]]] == \
                orule["gids"].items()
            ps = scheds[r]
            assert (ps.kind, ps.second, ps.minute, ps.hour, ps.dom, ps.month, ps.dow, ps.delay_ns) == \
                (osch.kind, osch.spec.second, osch.spec.minute, osch.spec.hour, osch.spec.dom,
                 osch.spec.month, osch.spec.dow, osch.delay_ns)
            r += 1
    assert r == js.n_rules
    # groups: membership as interned
    for _, og in ogroups:
        gi = [i for i in range(js.n_groups) if js.group_id(i) == og["id"]]
        assert len(gi) == 1
        g = gi[0]
        assert rin.group_exists[g]
        assert [lib_node(js, int(x)) for x in rin.group_nodes[rin.group_off[g]:rin.group_off[g + 1]]] \
            == og["nids"].items()
    return js


def lib_node(js, i):
    from cronsun_amd._lib import lib
    return lib().cg_jobset_node_id(js._h, i)


J = json.dumps


def test_basic_and_statuses():
    docs = [
        J({"id": "a", "name": "x", "rules": [{"id": "r1", "timer": "0 * * * * *", "gids": ["g1"],
                                              "nids": ["n1", "n2"], "exclude_nids": ["n2"]}],
           "kind": 1, "avg_time": 1500, "parallels": 9}),
        b"{bad json",
        J({"id": "b", "rules": [{"id": "r", "timer": ""}]}),            # ErrNilRule
        J({"id": "c", "rules": [{"id": "r", "timer": "61 * * * * *"}]}),  # parse error
        J({"id": "d", "rules": [None]}),                                  # nil rule: panic
        J({"id": "e", "kind": "1"}),                                      # type error
        J({"id": "a", "rules": [{"id": "r9", "timer": "@every 5s"}]}),    # replaces the first "a"
        b"null",                                                          # zero Job, ID ""
        b"[1,2]",                                                         # type error
        J({"id": "f", "avg_time": 1.5}),                                  # not an integer
        J({"id": "g", "timeout": 9223372036854775808}),                   # overflow
        J({"id": "h\u0000x"}),                                            # NUL in an ID
    ]
    js = _compare([d.encode() if isinstance(d, str) else d for d in docs],
                  [J({"id": "g1", "nids": ["n1", "n3"]}).encode(), b"{", J({"id": "g1", "nids": ["n9"]}).encode()])
    assert list(js.job_status) == [G.REPLACED, G.UNMARSHAL, G.INVALID, G.INVALID, G.PANIC, G.UNMARSHAL,
                                   G.OK, G.OK, G.UNMARSHAL, G.UNMARSHAL, G.UNMARSHAL, G.UNSUPPORTED]
    assert list(js.group_status) == [G.REPLACED, G.UNMARSHAL, G.OK]


def test_encoding_json_rules():
    docs = [
        # key folding: exact, ASCII case-insensitive, Kelvin sign / long s
        b'{"ID":"k1","Rules":[{"Id":"r","TIMER":"@hourly","NIDS":["x"]}],"KIND":1}',
        b'{"id":"k2","\xe2\x84\xaaind":2,"rule\xc5\xbf":[{"id":"r","timer":"@daily"}],"pau\xc5\xbfe":true}',
        b'{"id":"k3","avg_tim\xc5\xbf":5}',             # no s in avg_time: long s does not fold
        b'{"id":"k4","i\xc4\x91":"zz"}',                  # non-ASCII key: unknown field
        # duplicate keys: later wins; rules merge into the earlier *JobRule
        b'{"id":"d1","id":"d2","rules":[{"id":"a","timer":"@daily","nids":["1","2"]}],'
        b'"rules":[{"id":"b"}]}',
        # slice element reuse within capacity: the stale "2" reappears
        b'{"id":"s1","rules":[{"id":"r","timer":"@daily","nids":["1","2"],"nids":["x"],"nids":["y",null]}]}',
        # empty array drops the backing; null slice
        b'{"id":"s2","rules":[{"id":"r","timer":"@daily","nids":["1","2"],"nids":[],"nids":["y",null]}]}',
        b'{"id":"s3","rules":[{"id":"r","timer":"@daily","gids":null}],"to":null}',
        # null scalars are no-ops
        b'{"id":"n1","kind":1,"kind":null,"pause":true,"pause":null,"name":null}',
        # a rule element replaced by null then re-decoded
        b'{"id":"n2","rules":[{"id":"a","timer":"@daily"}],"rules":[null],"rules":[{"id":"b","timer":"@hourly"}]}',
        # escapes, surrogates, invalid UTF-8
        b'{"id":"e\\u00e9\\ud83d\\ude00\\ud800x\\/\\n","rules":[{"id":"\xff\xe2\x82z","timer":"@daily"}]}',
        # unknown fields of any type, nested
        b'{"id":"u1","extra":{"a":[1,{"b":null}],"c":"\\u0041"},"cnt":-0.5e-3}',
        # numbers: -0 ok, leading zero invalid JSON, exponent type error
        b'{"id":"x1","kind":-0}', b'{"id":"x2","kind":01}', b'{"id":"x3","kind":1e0}',
        # whitespace and trailing garbage
        b' \t\n{"id":"w1"}\r\n', b'{"id":"w2"} x', b'{"id":"w3",}',
        # control char in a string, bad escape
        b'{"id":"c1\x01"}', b'{"id":"c2\\q"}',
        # a rule that is not an object
        b'{"id":"t1","rules":["@daily"]}', b'{"id":"t2","rules":{"id":"r"}}',
        b'{"id":"t3","pause":"true"}', b'{"id":"t4","rules":[{"id":"r","timer":5}]}',
    ]
    _compare(docs)


def _random_doc(rng):
    def rid(p):
        return f"{p}{int(rng.integers(0, 40))}"
    timers = ["@every 10s", "0 */5 * * * *", "@daily", "1,2 * * * * ?", "* * *", "", "0 0 0 30 Feb ?",
              "@hourly", "*/7 * * * * *", "bad", "0 0 12 ? * MON-FRI"]
    job = {"id": rid("j"), "name": "n", "group": "grp", "cmd": "echo", "user": "u",
           "pause": bool(rng.random() < 0.2), "kind": int(rng.integers(0, 3)),
           "avg_time": int(rng.integers(-3000, 90000)), "parallels": int(rng.integers(0, 4)),
           "rules": []}
    for _ in range(int(rng.integers(0, 4))):
        job["rules"].append({"id": rid("r"), "timer": timers[int(rng.integers(0, len(timers)))],
                             "gids": [rid("g") for _ in range(int(rng.integers(0, 3)))],
                             "nids": [rid("n") for _ in range(int(rng.integers(0, 3)))],
                             "exclude_nids": [rid("n") for _ in range(int(rng.integers(0, 2)))]})
    b = J(job).encode()
    r = rng.random()
    if r < 0.15:  # flip a byte
        i = int(rng.integers(0, len(b)))
        b = b[:i] + bytes([int(rng.integers(0, 256))]) + b[i + 1:]
    elif r < 0.25:  # upper-case a key
        b = b.replace(b'"nids"', b'"NIDS"').replace(b'"timer"', b'"Timer"')
    elif r < 0.35:  # duplicate the rules key with a shorter array
        b = b[:-1] + b',"rules":[{"id":"z","timer":"@daily"}]}'
    elif r < 0.45:  # a type change
        b = b.replace(b'"pause": false', b'"pause": 0').replace(b'"kind": 1', b'"kind": "1"')
    elif r < 0.5:  # truncate
        b = b[:int(rng.integers(0, len(b)))]
    return b


def test_fuzzed_documents_match_oracle():
    rng = np.random.default_rng(20261016)
    docs = [_random_doc(rng) for _ in range(3000)]
    groups = [J({"id": f"g{i % 40}", "nids": [f"n{int(x)}" for x in rng.integers(0, 40, 3)]}).encode()
              for i in range(60)]
    js = _compare(docs, groups)
    st = np.array(js.job_status)
    # the mix exercises every outcome
    assert all((st == s).any() for s in (G.OK, G.UNMARSHAL, G.INVALID, G.REPLACED))


def test_ingest_feeds_the_schedule_and_node_paths():
    """The ingested set drives the same host resolution as the object model."""
    docs = [J({"id": "j1", "rules": [{"id": "r1", "timer": "@every 30s", "gids": ["g"], "nids": ["a"]}]}),
            J({"id": "j2", "pause": True, "rules": [{"id": "r2", "timer": "@daily", "nids": ["b"]}]})]
    js = _product([d.encode() for d in docs], [J({"id": "g", "nids": ["c"]}).encode()])
    assert js.is_run_on(0, "c") and js.is_run_on(0, "a") and not js.is_run_on(0, "b")
    assert js.cmds(1, "b") == []  # paused
    assert sorted(js.job_nodes(0)) == ["a", "c"]
