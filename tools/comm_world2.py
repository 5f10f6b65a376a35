"""The library's RCCL exchange at world > 1 on ONE GPU (a rehearsal of the
8-GPU node's multi-rank path, tests/test_gpu_comm.py::test_comm_world2_one_gpu).

RCCL refuses two ranks on one device of one host ("Duplicate GPU detected"),
so each rank here claims a host of its own (NCCL_HOSTID) and the ranks talk
over RCCL's socket transport on loopback.  The library code under test is the
same as on an 8-GPU node: cg_comm_init, cg_comm_allgather_i64,
cg_comm_node_offsets and cg_comm_gather_node_csr -- the status agreements,
the chunk plan, grouped ncclSend/ncclRecv per chunk, k_node_place /
k_span_place from the staging buffer and, for time-ordered results,
k_merge_ranks over the ranks' runs (cron.go:64-79,220 byTime order of every
node's Cron over every job, node/node.go:121-141).

  python3 tools/comm_world2.py <outdir> [world]      (the driver: starts the ranks)
  python3 tools/comm_world2.py <outdir> <world> <rank>  (one rank)

Rank r expands its job-ID range of a small multi-rule job set per node
(time order and rule order) and gathers it on a root through the library;
the root compares with the unsharded result of the same set computed by its
own engine, which the single-GPU tests hold against the oracle.  Every case
writes one JSON line to <outdir>/rank<r>.jsonl."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def driver(outdir, world):
    os.makedirs(outdir, exist_ok=True)
    procs = []
    for r in range(world):
        env = dict(os.environ)
        env["NCCL_HOSTID"] = f"cg-comm-rehearsal-{r}"  # one "host" per rank: no duplicate-GPU refusal
        env.setdefault("NCCL_SOCKET_IFNAME", "lo")
        env["NCCL_IB_DISABLE"] = "1"
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), outdir, str(world), str(r)], env=env))
    rcs = [p.wait(timeout=300) for p in procs]
    print("rank exit codes", rcs, flush=True)
    return 0 if all(rc == 0 for rc in rcs) else 1


def rank_main(outdir, world, rank):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from cronsun_amd import _lib, cron, synth
    from cronsun_amd.engine import Comm, Engine

    out = open(os.path.join(outdir, f"rank{rank}.jsonl"), "w")

    def emit(**kw):
        out.write(json.dumps(kw) + "\n")
        out.flush()

    uid_path = os.path.join(outdir, "uid.bin")
    if rank == 0:
        with open(uid_path + ".tmp", "wb") as f:
            f.write(Comm.unique_id())
        os.replace(uid_path + ".tmp", uid_path)
    t_end = time.time() + 60
    while not os.path.exists(uid_path):
        if time.time() > t_end:
            raise SystemExit("no unique id")
        time.sleep(0.05)
    uid = open(uid_path, "rb").read()
    eng = Engine(0)
    comm = Comm(eng, world, rank, uid)
    dev = torch.device("cuda", 0)
    emit(case="allgather", got=comm.allgather_i64([rank * 10 + 1, -rank]).tolist())

    rin = synth.multi_rule_jobs(3000, rules_per_job=(1, 3), n_nodes=97, n_groups=14, seed=31, key_choices=2)
    specs = synth.spec_mix(rin.n_rules, seed=32, mix=synth.MIX_CONFIG2)
    scheds = [cron.Parse(s) for s in specs]
    # job-ID-range shards cut at job boundaries (a job's rules stay together)
    starts = np.concatenate([[0], np.nonzero(np.diff(rin.rule_job))[0] + 1, [rin.n_rules]])
    cuts = [int(starts[np.argmin(np.abs(starts - rin.n_rules * g // world))]) for g in range(world)] + [rin.n_rules]
    lo, hi = cuts[rank], cuts[rank + 1]
    t0 = synth.T0_2026 + 3 * 86400
    t1 = t0 + 1800
    for order in (_lib.NODE_ORDER_TIME, _lib.NODE_ORDER_RULE):
        eng.set_node_order(order)
        ref = None
        if rank == 0 or rank == world - 1:  # the roots: the unsharded lists
            ref = eng.expand_per_node(scheds, None, t0, t1, rin, _lib.EXCLUDE_NONE)
        n_off, n_t, n_r = eng.expand_per_node(scheds[lo:hi], None, t0, t1, rin.slice_rules(lo, hi), _lib.EXCLUDE_NONE)
        start, base = comm.node_offsets(rin.n_nodes)
        if ref is not None:
            emit(case="node_offsets", order=int(order), ok=bool(np.array_equal(base, ref[0])))
        E = int(base[-1])
        peer_max = int(np.max(np.diff(base)))
        for root in sorted({0, world - 1}):
            for budget in (24 * world, 12 * max(2 * world, peer_max // 3), 1 << 30):
                if rank == root:
                    o = torch.empty(rin.n_nodes + 1, dtype=torch.int64, device=dev)
                    t = torch.full((E,), -1, dtype=torch.int64, device=dev)
                    r = torch.full((E,), -1, dtype=torch.int32, device=dev)
                    torch.cuda.synchronize(dev)
                    tg = time.perf_counter()
                    n = comm.gather_node_csr(root, lo, budget, o.data_ptr(), t.data_ptr(), r.data_ptr(), E)
                    dt = time.perf_counter() - tg
                    ok = (n == E and np.array_equal(o.cpu().numpy(), ref[0]) and np.array_equal(t.cpu().numpy(), ref[1])
                          and np.array_equal(r.cpu().numpy(), ref[2]))
                    emit(case="gather", order=int(order), root=root, budget=budget, events=E, ok=bool(ok),
                         seconds=dt)
                else:
                    comm.gather_node_csr(root, lo, budget)
    # time-ordered results whose rule bases descend with the rank: refused on
    # every rank before any transfer (the merge breaks ties by rank)
    eng.set_node_order(_lib.NODE_ORDER_TIME)
    eng.expand_per_node(scheds[lo:hi], None, t0, t1, rin.slice_rules(lo, hi), _lib.EXCLUDE_NONE)
    code = 0
    try:
        if rank == 0:
            o = torch.empty(rin.n_nodes + 1, dtype=torch.int64, device=dev)
            t = torch.empty(1 << 20, dtype=torch.int64, device=dev)
            r = torch.empty(1 << 20, dtype=torch.int32, device=dev)
            comm.gather_node_csr(0, 10**6 - lo, 1 << 30, o.data_ptr(), t.data_ptr(), r.data_ptr(), 1 << 20)
        else:
            comm.gather_node_csr(0, 10**6 - lo, 1 << 30)
    except _lib.CgError as e:
        code = e.code
    emit(case="descending_bases", code=int(code), expect=int(_lib.CG_EINVAL))
    # the communicator still works after the refusal
    emit(case="allgather_after", got=comm.allgather_i64([rank]).tolist())
    comm.free()
    eng.close()
    emit(case="done")


if __name__ == "__main__":
    if len(sys.argv) >= 4:
        rank_main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]))
    else:
        sys.exit(driver(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2))
