"""Debug helper: per-node lists vs oracle for one small case, first mismatch details."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import oracle_lib as O
from common import oracle_parse_all, oracle_zone, product_zone
from cronsun_amd import cron, synth
from cronsun_amd.engine import Engine

mode = int(sys.argv[1]) if len(sys.argv) > 1 else 2
eng = Engine(0)
rin = synth.multi_rule_jobs(300, seed=21)
specs = synth.spec_mix(rin.n_rules, seed=4, mix=synth.MIX_LIGHT)
scheds = [cron.Parse(s) for s in specs]
t0, t1 = synth.T0_2026 + 64 * 86400, synth.T0_2026 + 65 * 86400 + 3600
node_off, time, rule = eng.expand_per_node(scheds, product_zone("UTC"), t0, t1, rin, mode)
arr = O.sched_array(oracle_parse_all(specs))
eo, et = O.expand_batch(arr, t0, t1, oracle_zone("UTC"))
roff, rules = O.node_rules(rin, mode, np.arange(rin.n_nodes))
print("R", rin.n_rules, "E", eo[-1], "En", node_off[-1])
bad = 0
for n in range(rin.n_nodes):
    exp_t, exp_r = O.node_list(eo, et, rules[roff[n]:roff[n + 1]])
    got_t, got_r = time[node_off[n]:node_off[n + 1]], rule[node_off[n]:node_off[n + 1]]
    if len(got_t) != len(exp_t) or not (np.array_equal(got_t, exp_t) and np.array_equal(got_r, exp_r)):
        bad += 1
        if bad <= 3:
            m = min(len(got_t), len(exp_t))
            idx = np.nonzero((got_t[:m] != exp_t[:m]) | (got_r[:m] != exp_r[:m]))[0]
            print("node", n, "len", len(got_t), len(exp_t), "first bad", idx[:10], "node_off", node_off[n])
            for i in idx[:6]:
                r = int(exp_r[i])
                print("  i", i, "abs", node_off[n] + i, "got", int(got_t[i]), int(got_r[i]), "exp", int(exp_t[i]), r,
                      "rule fires", et[eo[r]:eo[r + 1]][:5], "got in rule?", int(got_t[i]) in set(et[eo[r]:eo[r+1]].tolist()))
print("bad nodes", bad)
