"""Debug: config 3 windows 0..3 through the pipelined per-node path vs the
synchronous per-node path vs the oracle, for a few nodes; reports the rules
whose fires differ.  python3 tools/debug_c3_window.py [order]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402
from cronsun_amd import _lib, cron, synth  # noqa: E402
from cronsun_amd.engine import Engine  # noqa: E402

order = sys.argv[1] if len(sys.argv) > 1 else "rule"
R = 1_000_000
HOUR = 3600
specs = synth.spec_mix(R, seed=0x5EED + 3, mix=synth.MIX_CONFIG2)
arr, status = cron.parse_batch(specs, threads=16)
rin = synth.rules_for_nodes(R, n_nodes=10_000, n_groups=500, seed=0x5EED + 3)
t0 = synth.T0_2026
eng = Engine(0)
sp = eng.upload_c(arr, R)
dr = eng.upload_rules(rin)
utc = cron.UTC()
E2, _ = eng.expand_per_node_rules_device(sp, utc, t0, t0 + 2 * HOUR, dr, 0)
print("sized E2", E2, flush=True)
if order == "time":
    eng.set_node_order(_lib.NODE_ORDER_TIME)
nodes = np.array([76, 1000, 5000], dtype=np.int32)
roff, nrules = O.node_rules(rin, 0, nodes, threads=16)
uniq = np.unique(nrules)
memo = {}
osch = O.sched_array([O.parse(specs[r])[0] for r in uniq])
loc = O.Loc("UTC")
off = np.empty(rin.n_nodes + 1, np.int64)
from cronsun_amd._lib import check, lib  # noqa: E402
for w in range(4):
    a, b = t0 + w * HOUR, t0 + (w + 1) * HOUR
    eo, et = O.expand_batch(osch, a, b, loc, threads=16)
    eng.expand_per_node_async(sp, utc, a, b, dr, 0)
    En = eng.expand_per_node_wait()
    check(lib().cg_node_result_copy(eng._h, off.ctypes.data, None, None, 0))
    res_async = {}
    for k, n in enumerate(nodes):
        res_async[n] = eng.node_copy_range(off[n], off[n + 1] - off[n])
    Es, _ = eng.expand_per_node_rules_device(sp, utc, a, b, dr, 0)
    offs = np.empty_like(off)
    check(lib().cg_node_result_copy(eng._h, offs.ctypes.data, None, None, 0))
    print(f"window {w}: async En {En} sync En {Es} offsets equal {np.array_equal(off, offs)}", flush=True)
    roff_rm, rt = eng.expand(sp, utc, a, b)
    for k, n in enumerate(nodes):
        rules = nrules[roff[k]:roff[k + 1]]
        pos = np.searchsorted(uniq, rules)
        exp_t, exp_p = O.node_list(eo, et, pos)
        exp_r = uniq[exp_p]
        st_t, st_r = eng.node_copy_range(offs[n], offs[n + 1] - offs[n])
        as_t, as_r = res_async[n]
        if order == "time":
            o = np.argsort(exp_t, kind="stable")
            exp_t, exp_r = exp_t[o], exp_r[o]
        ok_s = len(st_t) == len(exp_t) and np.array_equal(st_t, exp_t) and np.array_equal(st_r, exp_r)
        ok_a = len(as_t) == len(exp_t) and np.array_equal(as_t, exp_t) and np.array_equal(as_r, exp_r)
        print(f"  node {n}: exp {len(exp_t)} sync {len(st_t)} ok {ok_s} async {len(as_t)} ok {ok_a}", flush=True)
        if not (ok_s and ok_a):
            # per rule counts
            ce = {int(r): int(c) for r, c in zip(*np.unique(exp_r, return_counts=True))}
            for name, rr in (("sync", st_r), ("async", as_r)):
                cg = {int(r): int(c) for r, c in zip(*np.unique(rr, return_counts=True))}
                diff = [(r, ce.get(r, 0), cg.get(r, 0)) for r in set(ce) | set(cg) if ce.get(r, 0) != cg.get(r, 0)]
                print(f"    {name}: {len(diff)} rules differ, e.g. {diff[:8]}", flush=True)
                for r, c1, c2 in diff[:4]:
                    rm = rt[roff_rm[r]:roff_rm[r + 1]]
                    print(f"      rule {r} spec {specs[r]!r} oracle {c1} gpu-node {c2} gpu-rule-major {len(rm)}",
                          flush=True)
