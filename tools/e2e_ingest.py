"""End to end from cronsun's etcd values to per-node fire lists on one MI355X
("so that 10M-rule end-to-end runs are not host-bound").

  python tools/e2e_ingest.py [--jobs N] [--threads T]

Synthetic etcd values (config-3 shape: one rule per job, 0-3 group IDs, 0-4
node IDs, 0-2 excludes over 10k nodes / 500 groups, the light spec mix) are
generated first (not timed), then timed: bulk ingestion (JSON decode,
Job.Valid incl. cron.Parse, interning; host C++), upload of the schedules and
the interned rule set to HBM, one per-node expansion over 1 h, the batch
lockTtl of every rule and a dispatcher start + one wake.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    import numpy as np

    from cronsun_amd import cron, synth
    from cronsun_amd.engine import Engine
    from cronsun_amd.ingest import EtcdJobSet

    n = args.jobs
    rng = np.random.default_rng(0xE2E)
    t = time.perf_counter()
    specs = synth.spec_mix(n, seed=0xE2E, mix=synth.MIX_LIGHT)
    ng = rng.integers(0, 4, n)
    nn = rng.integers(0, 5, n)
    ne = rng.integers(0, 3, n)
    docs = []
    for i in range(n):
        docs.append(json.dumps({
            "id": f"job{i:08d}", "name": f"job {i}", "group": "default", "cmd": "/usr/bin/true",
            "user": "", "pause": bool(i % 100 == 0), "timeout": 0, "parallels": 0, "retry": 0,
            "interval": 0, "kind": int(i % 3), "avg_time": int(i % 5000), "fail_notify": False,
            "to": [],
            "rules": [{"id": f"r{i:08d}", "timer": specs[i],
                       "gids": [f"g{int(x)}" for x in rng.integers(0, 500, ng[i])],
                       "nids": [f"node{int(x)}" for x in rng.integers(0, 10000, nn[i])],
                       "exclude_nids": [f"node{int(x)}" for x in rng.integers(0, 10000, ne[i])]}]},
            separators=(",", ":")).encode())
        if i % 200_000 == 0:
            print(f"generated {i}", file=sys.stderr, flush=True)
    groups = [json.dumps({"id": f"g{g}", "name": f"group {g}",
                          "nids": [f"node{int(x)}" for x in rng.integers(0, 10000, rng.integers(4, 256))]}
                         ).encode() for g in range(500)]
    gen_s = time.perf_counter() - t
    mb = sum(len(d) for d in docs) / 1e6

    eng = Engine(0)
    utc = cron.UTC()
    out = {"jobs": n, "json_mb": mb, "threads": args.threads, "generate_s_untimed": gen_s}
    t = time.perf_counter()
    js = EtcdJobSet(docs, groups, threads=args.threads)
    out["ingest_s"] = time.perf_counter() - t
    out["ingested_jobs"] = int((js.job_status == 0).sum())
    t = time.perf_counter()
    sp = eng.upload_c(js.schedules_c(), js.n_rules)
    drules = eng.upload_rules(js.rules_in())
    eng.sync()
    out["upload_s"] = time.perf_counter() - t
    t0 = synth.T0_2026
    eng.expand_per_node_rules_device(sp, utc, t0, t0 + 3600, drules)  # warm
    eng.sync()
    t = time.perf_counter()
    En, nnz = eng.expand_per_node_rules_device(sp, utc, t0, t0 + 3600, drules)
    eng.sync()
    out["per_node_expand_s"] = time.perf_counter() - t
    out["node_events"], out["rule_node_pairs"] = En, nnz
    t = time.perf_counter()
    ttl = js.lock_ttls(t0, utc, 300, engine=eng)
    out["lock_ttl_s"] = time.perf_counter() - t
    out["lock_ttl_zero_rules"] = int((ttl == 0).sum())
    t = time.perf_counter()
    d = eng.dispatcher(sp, utc, t0)
    out["dispatcher_start_s"] = time.perf_counter() - t
    t = time.perf_counter()
    n_due, _ = d.fire_count(d.effective)
    out["dispatcher_wake_s"] = time.perf_counter() - t
    out["due_first_wake"] = n_due
    out["ingest_jobs_per_s"] = n / out["ingest_s"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
