"""Benchmark: fire events materialised/sec for BASELINE.json config 2
(1M mixed cron rules x 24 h horizon, UTC) per MI355X, weak-scaled over
job-ID-range shards at N > 1.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload W]
  (N > 1: one rank per GPU over RCCL.  Run under torch.distributed.run, or
  alone: `--gpus N` then starts torch.distributed.run with N ranks of the same
  command as a child process, before this process touches the GPU, and
  forwards rank 0's JSON line and the child's exit status.  A WORLD_SIZE that
  differs from --gpus is refused.)

At N > 1 every workload ends, after its timed region, with one verified
time-ordered per-node gather (`verify.gather`): a small pernode-shaped window
gathered on rank 0 in many chunks under a small byte budget (split nodes
included) -- through the library's RCCL communicator
(cg_comm_gather_node_csr: send/recv, placement, the merge of the ranks' runs)
with the nccl backend, through shard.gather_node_csr with gloo -- and 24 nodes
checked against the oracle.  With nccl the per-step exchanges (config-2
totals, per-node counts) also go through the library's communicator
(cg_comm_allgather_i64 / cg_comm_node_offsets; `--torch-comm`: through
torch.distributed instead).

Workloads (`--workload`, default config2 -- the headline line):
  config2  a step = one full expansion of the rank's 1M-rule shard over 24 h:
           count -> scan -> slice map -> closed-form write -> walk write ->
           offsets, specs resident in HBM, fire times left in HBM.  At N > 1
           each step also all-gathers the per-rank event totals (global CSR
           offsets) over RCCL.
  pernode  config 3 shape: 1M jobs x 10k nodes (500 groups, 0-3 GroupIDs,
           0-4 NodeIDs, 0-2 ExcludeNodeIDs per rule), the lighter spec mix and
           a 1 h horizon so the per-node fan-out fits HBM; a step = expansion +
           rule->node join + transpose + per-node (time, rule) lists, rules
           resident in HBM (cg_rules_upload).  At N > 1 the per-node counts are
           all-gathered over RCCL (per-node offsets of every rank's slice).
  config4  config 4 shape: 10M rules x 7 days over the job-ID-range shards of
           N GPUs (10M / N rules per rank, lighter spec mix); a step = one
           expansion per rank.  Fixed total work: `scaling` = "strong".
           With --per-node (north_star's target, "per-node fire schedules for
           10M rules x 7-day horizon"): config 3's node model (10k nodes, 500
           groups) over the config-4 rule set, per-node lists of the rank's
           job-ID range streamed in pipelined windows (`--window`, default
           90 min for a rank of > 5M rules, else 1 h; 30 min in time order past
           2^20 rules; a window's lists fit HBM); a step = the whole 7 days; the per-node counts of every
           window all-gathered at N > 1 (cg_comm_node_offsets with --lib-comm).
  config3  config 3 as specified: 1M jobs x 10k nodes, the config-2 spec mix,
           24 h -> per-node lists, streamed in 1 h windows (`--window`; the
           whole day's 62 G node events would not fit one GPU's HBM): a step
           = 24 windows of expansion + join + transpose + per-node write, each
           window's per-node counts all-gathered at N > 1.  `--exclude-mode`
           none (the scheduling path) | rule | cumulative (web/job.go).
  dispatch SURVEY.md §8(f)-1: Cron.run's entry table resident in HBM, 10M
           entries of the config-2 mix per GPU; a step = one on-time wake
           (fire every entry whose Next is the earliest, Next(now) for them,
           next minimum, ordered due list left in HBM).

Prints one JSON line (rank 0).  See DESIGN.md §Measurement for the roofline
and CPU-baseline definitions.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
SPEC_BYTES = 32          # packed spec per rule in HBM
METRIC = "fire events materialised/sec (1M rules × 24h) + HBM GB/s at 1/2/4/8 GPU"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(tag, rules, events, kernels, per, scale=1, windows=None):
    """HBM bytes of one timed interval, from the newest committed rocprofv3
    PMC summary profiles/rNN_pmc_traffic[_<tag>][_vK].json (written by
    tools/pmc_traffic.py from FETCH_SIZE / WRITE_SIZE passes) measured on the
    same workload -- same tag (workload and list order), rules and events per
    step: the bytes of every launch of the kernels named by the `kernels`
    prefixes, per launch of `per` (e.g. a pipelined window's writer plus its
    time-order pass), times `scale` (the windows of a step).  None when no
    such profile is committed."""
    import glob
    import re
    pat = re.compile(r"r\d+_pmc_traffic" + (("_" + re.escape(tag)) if tag else "") + r"(_v\d+)?\.json$")
    paths = [p for p in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic*.json"))
             if pat.search(os.path.basename(p))]

    def key(p):  # newest round, then newest version
        m = re.search(r"r(\d+)_.*?(?:_v(\d+))?\.json$", os.path.basename(p))
        return (int(m.group(1)), int(m.group(2) or 0))
    for path in sorted(paths, key=key, reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
            if d.get("rules") != rules or d.get("events") != events:
                continue
            if windows is not None and d.get("windows", windows) != windows:
                continue  # another windowing of the same step: other bytes per launch
            ks = d["kernels"]
            n_per = ks[per]["calls"]
            tot = sum(v["hbm_bytes_per_launch"] * v["calls"] for k, v in ks.items()
                      if k.startswith(tuple(kernels)) and "hbm_bytes_per_launch" in v)
            return {"bytes": tot / n_per * scale, "profile": os.path.relpath(path, ROOT),
                    "kernels": sorted(k for k in ks if k.startswith(tuple(kernels)))}
        except Exception:
            pass
    return None


def store_ceiling(eng, nbytes, dev, achieved_gbps, reps=5):
    """Store rate of `nbytes` of HBM on this box, beside the 8 TB/s nominal
    peak (outside the timed region): the production library's streaming fill
    (k_fill_stream: 16 B per lane, one launch over the buffer, nontemporal and
    plain stores) and hipMemsetAsync, each timed with HIP events on the
    library's stream (cg_fill_rate_device, mean of `reps` after a warm-up).
    The output-bound kernel's achieved rate is reported as a fraction of the
    fastest of the three."""
    import torch
    nbytes = nbytes // 16 * 16
    buf = torch.empty(nbytes // 8, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    ms = eng.fill_rates(buf.data_ptr(), nbytes, reps)
    del buf
    torch.cuda.empty_cache()
    rates = {k: nbytes / v / 1e6 for k, v in ms.items() if v > 0}
    best = max(rates, key=rates.get)
    return {"kind": "fastest of k_fill_stream (16 B/lane nt | plain stores, one 4-wave block per CU, one launch) and "
                    "hipMemsetAsync over the kernel's output bytes", "bytes": nbytes,
            "ms": ms, "GBps": rates, "best": best, "best_GBps": rates[best],
            "frac_of_ceiling": achieved_gbps / rates[best]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["config2", "pernode", "config3", "config4", "dispatch", "parse"],
                    default="config2")
    ap.add_argument("--rules", type=int, default=0, help="rules per GPU (0 = the workload's)")
    ap.add_argument("--horizon", type=int, default=0, help="seconds (0 = the workload's)")
    ap.add_argument("--window", type=int, default=0,
                    help="per-node output window in seconds (0 = the workload's; config3: 3600)")
    ap.add_argument("--exclude-mode", choices=["none", "rule", "cumulative"], default="none")
    ap.add_argument("--zone", default="UTC",
                    help="time zone of the expansion (UTC, or a TZif name under tests/golden/zoneinfo, "
                         "e.g. America/New_York: the walk path near DST transitions)")
    ap.add_argument("--t0", type=int, default=0,
                    help="horizon start, unix seconds (0 = the workload's: 2026-01-05T00:00Z)")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="rules in the CPU-baseline sample (0 = skip; default 40k, 1M for dispatch)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--verify-sample", type=int, default=2000,
                    help="rules (rule-major) or nodes/250 (per-node) of the timed result checked "
                         "against the oracle after the timed region (0 = skip)")
    ap.add_argument("--gather-node-csr", action="store_true",
                    help="pernode/config3 at N > 1: every step also gathers the whole per-node CSR on "
                         "rank 0 (shard.gather_node_csr; timed)")
    ap.add_argument("--lib-comm", action="store_true",
                    help="N > 1: the exchanges through the library's RCCL communicator behind the C-ABI "
                         "(cg_comm_*: totals all-gather, per-node offsets, chunked per-node CSR gather); "
                         "the default with the nccl backend")
    ap.add_argument("--torch-comm", action="store_true",
                    help="N > 1 with nccl: the per-step exchanges through torch.distributed instead of "
                         "the library's communicator")
    ap.add_argument("--no-gather-check", action="store_true",
                    help="N > 1: skip the verified time-ordered per-node gather after the timed region")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check: every rank reports its rank / world and exits before any GPU use")
    ap.add_argument("--gather-budget", type=int, default=1 << 31,
                    help="bytes of peer events rank 0 stages per chunk of the per-node CSR gather")
    ap.add_argument("--sync", action="store_true",
                    help="config2/config4: synchronous steps (cg_expand_device: every step ends with a "
                         "stream sync) instead of the pipelined cg_expand_device_async")
    ap.add_argument("--tick", type=int, default=0,
                    help="config2/config4: advance T0 (and T1) by this many seconds every step, as a "
                         "scheduler's consecutive windows (0 = the same window every step)")
    ap.add_argument("--per-node", action="store_true",
                    help="config4: per-node lists over config 3's node model (north_star's 10M x 7 d "
                         "per-node target) instead of the rule-major CSR")
    ap.add_argument("--time-order", action="store_true",
                    help="pernode/config3: every window's per-node lists in (time, rule) order "
                         "(cg_set_node_order(TIME): the order pass inside every per-node call, pipelined)")
    ap.add_argument("--order-pass", action="store_true",
                    help="with --time-order: rule-major lists reordered afterwards by "
                         "cg_node_result_order_by_time (the separate pass; synchronous windows)")
    ap.add_argument("--diagnostic", action="store_true",
                    help="allow the diagnostic library / CG_WRITE_* CG_NODE_* switches (the line is "
                         "then marked diagnostic and is not a headline)")
    args = ap.parse_args()

    if args.workload == "parse":  # host-only: no GPU, no ranks
        print(json.dumps(parse_line(args)), flush=True)
        return
    rc = launch_ranks(args)  # before anything touches torch.cuda, HIP or the library
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and os.environ.get("CG_RCCL_ONE_GPU_REHEARSAL"):
        # rehearsal of the N-GPU RCCL path with N ranks on fewer GPUs: RCCL
        # refuses two ranks on one device of one host, so every rank claims a
        # host of its own and RCCL moves the data over sockets on loopback
        # (tools/comm_world2.py does the same for the library's gather)
        os.environ["NCCL_HOSTID"] = f"cg-bench-rank-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ["NCCL_IB_DISABLE"] = "1"
    if args.dry_run:
        if rank == 0:
            print(json.dumps({"dry_run": True, "rank": rank, "world": world, "gpus": args.gpus}), flush=True)
        return
    import numpy as np
    import torch
    import torch.distributed as dist

    # A headline must come from the production library with every output
    # store in place: the diagnostic build's probe/variant switches replace or
    # drop stores (cronsun_amd/csrc/Makefile `diag`).
    from cronsun_amd import _lib as _cg
    diag_env = {k: v for k, v in os.environ.items() if k.startswith(("CG_WRITE_", "CG_NODE_"))}
    build_info = _cg.lib().cg_build_info()
    if (diag_env or build_info & 1) and not args.diagnostic:
        log(f"bench.py: refusing to run: diagnostic switches {sorted(diag_env)} / library build "
            f"info {build_info} ({_cg.LIB_PATH}); pass --diagnostic for a non-headline probe run")
        sys.exit(2)
    # RCCL ("nccl") in production; CG_DIST_BACKEND=gloo rehearses the N > 1
    # path with several ranks sharing fewer GPUs (collectives on host tensors)
    backend = os.environ.get("CG_DIST_BACKEND", "nccl")
    ndev = max(torch.cuda.device_count(), 1)
    if world > 1:
        local = local % ndev
        torch.cuda.set_device(local)
        dist.init_process_group(backend)

    from cronsun_amd import cron, shard, synth
    from cronsun_amd.engine import Engine
    cdev_early = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")

    wl = args.workload
    if args.cpu_sample is None:  # config2: -1 = adaptive (the whole workload when it fits ~30 s)
        args.cpu_sample = 1_000_000 if wl == "dispatch" else -1
    if wl == "config2":
        R = args.rules or 1_000_000  # per GPU (weak scaling): the global set has R * world rules
        H = args.horizon or 86400
        mix = synth.MIX_CONFIG2
        seed = 0x5EED
    elif wl == "dispatch":
        R = args.rules or 10_000_000
        H = 0
        mix = synth.MIX_CONFIG2
        seed = 0x5EED + 5 + rank
    elif wl == "pernode":
        R = args.rules or 1_000_000  # per GPU: the global set has R * world jobs
        H = args.horizon or 3600
        mix = synth.MIX_LIGHT
        seed = 0x5EED + 3
    elif wl == "config3":
        R = args.rules or 1_000_000
        H = args.horizon or 86400
        mix = synth.MIX_CONFIG2
        seed = 0x5EED + 3
    else:  # config4: 10M rules in total, job-ID-range shards balanced by events
        total = args.rules or 10_000_000
        R = total
        H = args.horizon or 7 * 86400
        mix = synth.MIX_LIGHT
        seed = 0x5EED + 4
    t0 = args.t0 or synth.T0_2026
    t1 = t0 + H
    if args.per_node and wl != "config4":
        ap.error("--per-node applies to --workload config4 (pernode/config3 are per-node already)")
    pn = wl in ("pernode", "config3") or args.per_node
    W = args.window or (3600 if wl == "config3" else H)
    xmode = {"none": 0, "rule": 1, "cumulative": 2}[args.exclude_mode]
    eng = Engine(local)
    if args.zone == "UTC":
        utc = cron.UTC()
    else:  # the committed tzdata (the GPU box has no other zoneinfo guarantee)
        with open(os.path.join(ROOT, "tests", "golden", "zoneinfo", args.zone), "rb") as f:
            utc = cron.LoadLocationFromTZData(args.zone, f.read())
    log(f"[rank {rank}] {wl}: generating {R} rules")
    shard_info = None
    if wl == "config4":
        # the global 10M-rule set is the 1M-rule light-mix block tiled in
        # job-ID order (rule i = block[i % 1M]), so any rank can build any range
        base_n = min(total, 1_000_000)
        base_specs = synth.spec_mix(base_n, seed=seed, mix=mix)
        base_arr, status = cron.parse_batch(base_specs, threads=16)
        assert (status == 0).all()
        base_np = np.ctypeslib.as_array(base_arr)

        def upload_range(lo, hi):
            a = np.ascontiguousarray(base_np[np.arange(lo, hi) % base_n])
            return eng.upload_c((base_arr._type_ * (hi - lo)).from_buffer(a), hi - lo)

        if world > 1:
            # §8e: a cheap count pass over a provisional equal slice, one
            # all-gather of per-block event sums, cuts of equal estimated events
            tc = time.perf_counter()
            lo, hi, _ = shard.event_balanced_range(
                total, lambda a, b: eng.count(upload_range(a, b), utc, t0, t1), dist,
                block=65536, device=cdev_early)
            shard_info = {"lo": lo, "hi": hi, "count_pass_s": time.perf_counter() - tc}
        else:
            lo, hi = 0, total
        R = hi - lo
        sp = upload_range(lo, hi)
        specs = None
        shard_lo = lo
        if shard_info is None:
            shard_info = {"lo": lo, "hi": hi}
        shard_info["global_rules"] = total
        if pn and not args.window:
            # 90-min windows for a rank of > 5M rules (10M: ~14.5 G node events,
            # 173 GB of lists, within HBM beside the three window sets'
            # records), else 1 h: the per-window side chain (rule infos,
            # segment records over all ~930 M pairs, ~8.4 ms) is paid 112 times
            # per step instead of 168 (336 at 30 min): 5.16 vs 5.37 s per step
            # on one box, 80 min 5.35 (profiles/r06_ab_config4pn_windows.txt).
            # Time order past 2^20 rules per rank keeps 30-min windows: their
            # 32-s slabs fit k_ot_mid's chunks (64-s slabs of a 1-h window
            # would go to k_ot_big's two reads).  2048-s windows (64 slabs of
            # 32 s, 296 windows) measured the same: 15.56 vs 15.49 s per step,
            # more slabs past k_ot_mid's chunk (profiles/r06_pmc_traffic_config4pn_order_2048.json)
            W = 1800 if (args.time_order and R > (1 << 20)) else (5400 if R > 5_000_000 else 3600)

        def spec_of(i):  # local rule i of this rank's range
            return base_specs[(shard_lo + i) % base_n]
    elif wl in ("config2", "pernode", "config3"):
        # one global rule set of R * world rules in job-ID order, built from
        # R-rule blocks (block b: seed 0x5EED + b, so the N = 1 set is block 0);
        # rank g expands its job-ID range [g R, (g + 1) R)
        glob = R * world
        lo, hi = shard.shard_range(glob, world, rank)
        specs = []
        for b in range(lo // R, (hi - 1) // R + 1):
            blk = synth.spec_mix(R, seed=seed + b, mix=mix)
            specs += blk[max(lo - b * R, 0):min(hi - b * R, R)]
        shard_info = {"lo": lo, "hi": hi, "global_rules": glob}
        arr, status = cron.parse_batch(specs, threads=16)
        assert (status == 0).all()
        sp = eng.upload_c(arr, R)
    else:
        if wl == "dispatch" and R > 1_000_000:
            # the 1M-rule config-2 set tiled (Python generation of 10M strings
            # takes minutes; entries are independent, so repeats change nothing)
            base = synth.spec_mix(1_000_000, seed=seed, mix=mix)
            specs = (base * (R // len(base) + 1))[:R]
        else:
            specs = synth.spec_mix(R, seed=seed, mix=mix)
        arr, status = cron.parse_batch(specs, threads=16)
        assert (status == 0).all()
        sp = eng.upload_c(arr, R)
    if specs is not None:
        def spec_of(i):
            return specs[i]
    drules = None
    n_nodes = 10_000
    if pn:
        # the global jobs x groups x nodes set (one rule per job), this rank's
        # job-ID range of it (the same 500 groups and 10k nodes everywhere)
        if wl == "config4":
            rin = synth.rules_for_nodes(total, n_nodes=n_nodes, n_groups=500, seed=0x5EED + 4)
        else:
            rin = synth.rules_for_nodes(R * world, n_nodes=n_nodes, n_groups=500, seed=0x5EED + 3)
        if world > 1:
            rin = rin.slice_rules(shard_info["lo"], shard_info["hi"])
        drules = eng.upload_rules(rin)

    def barrier():
        if world > 1:
            dist.barrier()

    dev = torch.device("cuda", local)
    cdev = dev if backend == "nccl" else torch.device("cpu")  # collective tensors
    lcomm = None
    if world > 1 and (args.lib_comm or (backend == "nccl" and not args.torch_comm)):
        # the library's own RCCL communicator (cg_comm_init): rank 0's unique id
        # handed to every rank over torch.distributed
        from cronsun_amd.engine import Comm
        uid = [Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        lcomm = Comm(eng, world, rank, uid[0])
    gath = {}
    tot = torch.zeros(world, dtype=torch.int64, device=cdev)
    node_counts = torch.zeros(n_nodes, dtype=torch.int64, device=dev) if pn else None
    last = {}

    disp = eng.dispatcher(sp, utc, t0) if wl == "dispatch" else None
    wake = {"due": 0, "wakes": 0}

    def step():
        if wl == "dispatch":
            tw = time.perf_counter()
            n_due, _ = disp.fire_count(disp.effective)  # an on-time wake
            wake.setdefault("wall", []).append(time.perf_counter() - tw)
            wake["due"] += n_due
            wake["wakes"] += 1
            return n_due
        if pn and pn_pipelined and last.get("pn_sized"):
            # pipelined windows, enqueued: window k+1's expansion and records
            # overlap window k's per-node writer, across steps too (a tick
            # loop); finish() waits once (the node events of every window come
            # with it)
            wins = list(range(t0, t1, W))
            s_no = last.get("timed_no")
            for i, a in enumerate(wins):
                eng.expand_per_node_async(sp, utc, a, min(a + W, t1), drules, xmode)
                if s_no is not None and i == ck["win"][s_no]:
                    # the seeded window of this timed step: checksums of the
                    # sample nodes' lists, enqueued right behind its writer
                    eng.node_checksum_enqueue(ck["nodes"].data_ptr(), len(ck["nodes"]), ck["out"][s_no].data_ptr())
            if s_no is not None:
                last["timed_no"] = s_no + 1
            last["pending_steps"] = last.get("pending_steps", 0) + 1
            last["windows"] = len(wins)
            return None
        if pn:
            En = 0
            kt_sum = np.zeros(6)
            nkt_sum = np.zeros(3)
            for a in range(t0, t1, W):  # per-node lists window by window
                En_w, nnz = eng.expand_per_node_rules_device(sp, utc, a, min(a + W, t1), drules,
                                                             xmode)
                En += En_w
                last["En_last"] = En_w
                kt_sum += np.array(eng.kernel_times())
                nkt_sum += np.array(eng.node_kernel_times())
                if args.time_order:  # the pass's time: run here, or inside the per-node call
                    last["order_ms"] = last.get("order_ms", 0.0) + (
                        eng.node_order_by_time() if args.order_pass else eng.last_order_ms())
                last.setdefault("first_nkt", eng.node_kernel_times())  # the uncached join
                if world > 1 and args.gather_node_csr and lcomm is not None:
                    # the gather behind the C-ABI (cg_comm_gather_node_csr):
                    # node-range chunks under the byte budget, RCCL send/recv
                    if rank == 0 and not gath:
                        cap = 2 * En_w * world + (1 << 20)  # every window about the same size
                        gath.update(off=torch.empty(rin.n_nodes + 1, dtype=torch.int64, device=dev),
                                    t=torch.empty(cap, dtype=torch.int64, device=dev),
                                    r=torch.empty(cap, dtype=torch.int32, device=dev), cap=cap)
                    ptrs = (gath["off"].data_ptr(), gath["t"].data_ptr(), gath["r"].data_ptr(), gath["cap"]) \
                        if rank == 0 else (0, 0, 0, 0)
                    last["gathered_events"] = lcomm.gather_node_csr(0, shard_info["lo"], args.gather_budget,
                                                                    *ptrs)
                elif world > 1 and args.gather_node_csr:
                    # north_star's second collective: the whole per-node CSR on
                    # rank 0 (per-node counts all-gathered, then each rank's
                    # slice to rank 0 over its own link, in chunks under the budget)
                    n_off, n_time, n_rule = eng.node_result_tensors(rin.n_nodes)
                    g = shard.gather_node_csr(n_off.to(cdev), n_time.to(cdev), n_rule.to(cdev),
                                              shard_info["lo"], dist, engine=eng, budget_bytes=args.gather_budget,
                                              order="time" if args.time_order else "rule")
                    if g is not None:
                        last["gathered_events"] = int(g[1].numel())
                    del g
                elif lcomm is not None:
                    lcomm.node_offsets(rin.n_nodes)  # per-node offsets over the library's RCCL comm
                elif world > 1:
                    # per-node offsets of every rank's slice (RCCL allgather of N int64)
                    eng.node_counts_to_device(node_counts.data_ptr())
                    shard.node_offsets(node_counts.to(cdev), dist)
            last.update(nnz=nnz, kt=kt_sum, nkt=nkt_sum, windows=len(range(t0, t1, W)), pn_sized=True,
                        kt_sync=kt_sum, nkt_sync=nkt_sum)
            return En
        off_t = args.tick * last.get("step_no", 0)
        last["step_no"] = last.get("step_no", 0) + 1
        last["window"] = (t0 + off_t, t1 + off_t)
        if pipelined:
            # enqueued; the pipeline's results and errors come with expand_wait
            eng.expand_async(sp, utc, t0 + off_t, t1 + off_t)
            return None
        E = eng.expand_device(sp, utc, t0 + off_t, t1 + off_t)
        if lcomm is not None:
            lcomm.allgather_i64([E])  # global CSR offsets over the library's RCCL comm
        elif world > 1:
            # global CSR offsets of the job-ID-range shards (RCCL allgather)
            mine = torch.tensor([E], dtype=torch.int64, device=cdev)
            dist.all_gather_into_tensor(tot, mine)
        return E

    def finish():
        """End of a run of steps: drain the pipeline (pipelined mode); at N > 1
        one allgather of the ranks' totals gives the shards' global offsets
        (per-node: of every rank's per-node counts of the last window).
        Returns the events of one step."""
        if pn and pn_pipelined and last.get("pending_steps"):
            En_w, En = eng.expand_per_node_wait(with_total=True)
            k = last.pop("pending_steps")
            last["En_last"] = En_w
            nk = eng.node_kernel_times()
            last.update(kt=np.array(last["kt_sync"]),
                        nkt=np.array([last["nkt_sync"][0], last["nkt_sync"][1], nk[2] * last["windows"]]))
            if lcomm is not None:
                lcomm.node_offsets(rin.n_nodes)
            elif world > 1:
                eng.node_counts_to_device(node_counts.data_ptr())
                shard.node_offsets(node_counts.to(cdev), dist)
            return En // k
        if not pipelined:
            return None
        E = eng.expand_wait()
        if lcomm is not None:
            lcomm.allgather_i64([E])
        elif world > 1:
            mine = torch.tensor([E], dtype=torch.int64, device=cdev)
            dist.all_gather_into_tensor(tot, mine)
        return E

    # Throughput runs time k_write_cf only (HIP events around it); an event
    # between every phase leaves the GPU idle for several us per event.  The
    # other phases are timed afterwards, outside the timed region.
    lean = not pn and wl != "dispatch"
    pipelined = lean and not args.sync
    # per-node windows pipelined (cg_expand_per_node_rules_device_async) after
    # a synchronous warmup step sized the outputs; the time-order pass and the
    # gather need every window's result, so they keep synchronous windows
    pn_pipelined = pn and not args.sync and not args.order_pass and not args.gather_node_csr
    if pn and args.time_order and not args.order_pass:
        eng.set_node_order(_cg.NODE_ORDER_TIME)
    if pn_pipelined and args.warmup < 4:
        # one synchronous step sizes the outputs, then one pipelined step per
        # window set (3) so no set allocates its buffers inside the timed steps
        args.warmup = 4
    if lean:
        eng.set_phase_timing(1)
    if pipelined:  # a synchronous call sizes the output for the pipelined ones
        eng.expand_device(sp, utc, t0, t1 + args.tick * (args.warmup + args.steps + 8))
    for _ in range(args.warmup):
        E = step()
    if pipelined or pn_pipelined:
        E = finish() or E
    log(f"[rank {rank}] warmup done: {E} events/step ({'pipelined' if pipelined else 'synchronous'} steps)")
    if not pn and wl != "dispatch":
        _, d_times, _ = eng.result_device()
        log(f"[rank {rank}] times buffer at {d_times:#x} ({d_times % (1 << 21):#x} past a 2 MiB boundary)")
    # Poison the result buffers (outside the timed region): whatever a timed
    # step fails to write stays -1 and is counted after the timed loop.
    def result_buffers():
        if pn:
            _, d_time, d_rule, n_ev = eng.node_result_device()
            return [(d_time, n_ev, 8), (d_rule, n_ev, 4)]
        _, d_times, n_ev = eng.result_device()
        return [(d_times, n_ev, 8)]
    if wl != "dispatch":
        for ptr, n_ev, w in result_buffers():
            eng.fill(ptr, n_ev * w, 0xFF)
    # per-node pipelined steps: every timed step checks one seeded window (its
    # lists are overwritten by later windows) through device checksums of a
    # node sample, compared with the oracle after the timed region
    ck = None
    if pn_pipelined and args.verify_sample > 0:
        rng_ck = np.random.default_rng(0x5EED + 31 + rank)
        nw_ck = len(range(t0, t1, W))
        ck = {"nodes_np": np.sort(rng_ck.choice(n_nodes, 8, replace=False)).astype(np.int32),
              "win": rng_ck.integers(0, nw_ck, args.steps)}
        ck["nodes"] = torch.from_numpy(ck["nodes_np"]).to(dev)
        ck["out"] = torch.zeros((args.steps, 16), dtype=torch.int64, device=dev)
        last["timed_no"] = 0
    barrier()
    torch.cuda.synchronize()
    start = time.perf_counter()
    kts, nkts = [], []
    wake["due"] = wake["wakes"] = 0
    wake["wall"] = []
    step_wall = []
    last["order_ms"] = 0.0
    for _ in range(args.steps):
        ts = time.perf_counter()
        E = step()
        step_wall.append(time.perf_counter() - ts)
        if pn and not pn_pipelined:
            kts.append(last["kt"])
            nkts.append(last["nkt"])
        elif not pipelined and not pn:
            kts.append(eng.kernel_times())
            nkts.append(eng.dispatch_kernel_times() if wl == "dispatch" else eng.node_kernel_times())
    if pn_pipelined:  # inside the timed region: every window is done and checked
        E = finish()
        kts.append(last["kt"])
        nkts.append(last["nkt"])
    elif pipelined:  # inside the timed region: every step's work is done and checked
        E = finish()
        kts.append(eng.kernel_times())  # [3] = mean k_write_cf time of the timed steps
        nkts.append(eng.node_kernel_times())
    t_loop = time.perf_counter() - start
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - start
    wake["loop_s"], wake["tail_s"] = t_loop, elapsed - t_loop

    # The timed steps' own output, checked on a seeded sample against the
    # oracle (outside the timed region): a step that skipped work would fail.
    verify = None
    unwritten = None
    if wl != "dispatch":  # poisoned words the timed steps left unwritten (must be 0)
        unwritten = sum(eng.count_value(ptr, n_ev, w, -1) for ptr, n_ev, w in result_buffers())
    if args.verify_sample > 0 and wl != "dispatch":
        tv = time.perf_counter()
        if pn:
            a_last = list(range(t0, t1, W))[-1]
            verify = verify_per_node(eng, spec_of, rin, xmode, a_last, min(a_last + W, t1), last["En_last"],
                                     max(2, args.verify_sample // 250), seed=0x5EED + 77 + rank,
                                     zone=args.zone, time_order=args.time_order)
        else:
            wa, wb = last.get("window", (t0, t1))  # the last timed step's window
            verify = verify_rule_major(eng, spec_of, R, wa, wb, E, args.verify_sample,
                                       seed=0x5EED + 99 + rank, zone=args.zone)
        if ck is not None:
            verify["every_step"] = verify_window_checksums(eng, spec_of, rin, xmode, t0, t1, W, ck,
                                                           zone=args.zone, time_order=args.time_order)
            verify["verified"] = verify["verified"] and verify["every_step"]["verified"]
        verify["seconds"] = time.perf_counter() - tv
        verify["unwritten_after_poison"] = unwritten
        verify["verified"] = verify["verified"] and unwritten == 0
        ok = torch.tensor([1 if verify["verified"] else 0], dtype=torch.int64, device=cdev)
        if world > 1:
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        verify["verified_all_ranks"] = bool(ok.item())
        log(f"[rank {rank}] verify: {verify}")

    if world > 1 and not args.no_gather_check:
        # the multi-rank exchange itself, verified (outside the timed region)
        g = gather_check(eng, dist, world, rank, backend, utc, args.zone, t0, dev, cdev,
                         restore_order=_cg.NODE_ORDER_TIME if (pn and args.time_order) else _cg.NODE_ORDER_RULE)
        if rank == 0:
            log(f"[rank 0] gather check: {g}")
            if verify is None:
                verify = {"verified": True, "verified_all_ranks": True}
            verify["gather"] = g
            verify["verified_all_ranks"] = verify["verified_all_ranks"] and g["verified"]

    if lean:
        # per-phase breakdown of a few untimed steps (events between phases)
        eng.set_phase_timing(2)
        phases = []
        for _ in range(3):  # synchronous calls: one per step, events between all phases
            eng.expand_device(sp, utc, t0, t1)
            phases.append(eng.kernel_times())
        eng.set_phase_timing(1)
        ph = np.mean(np.array(phases), axis=0)
        kts = [[ph[0], ph[1], ph[2], k[3], ph[4], ph[5]] for k in kts]

    e2e = None
    if wl == "config2" and rank == 0:
        # end to end, outside the timed region: H2D of the
        # packed specs, the expansion, D2H of the rule-major CSR into pinned
        # host memory (the host parse is reported by the CPU baseline)
        from cronsun_amd._lib import check as _check, lib as _cglib
        host_times = torch.empty(E, dtype=torch.int64, pin_memory=True)
        host_off = torch.empty(R + 1, dtype=torch.int64, pin_memory=True)
        torch.cuda.synchronize()
        te = time.perf_counter()
        sp2 = eng.upload_c(arr, R)
        t_h2d = time.perf_counter() - te
        wa, wb = last.get("window", (t0, t1))  # the last timed step's window (E events)
        E2 = eng.expand_device(sp2, utc, wa, wb)
        t_exp = time.perf_counter() - te - t_h2d
        _check(_cglib().cg_result_copy_offsets(eng._h, host_off.data_ptr()))
        _check(_cglib().cg_result_copy_times(eng._h, 0, E2, host_times.data_ptr()))
        t_all = time.perf_counter() - te
        assert E2 == E and int(host_off[-1]) == E
        e2e = {"ms": t_all * 1e3, "h2d_specs_ms": t_h2d * 1e3, "expand_ms": t_exp * 1e3,
               "d2h_csr_ms": (t_all - t_h2d - t_exp) * 1e3,
               "d2h_gbps": (E + R + 1) * 8 / max(t_all - t_h2d - t_exp, 1e-9) / 1e9,
               "events_per_s": E / t_all}
        sp2.free()
        del host_times, host_off

    step_events = E * args.steps
    if args.tick and not pn and wl != "dispatch":
        # moving windows: every timed step's own total, counted afterwards
        # (outside the timed region) with the count pass alone
        step_events = sum(int(eng.count(sp, utc, t0 + args.tick * i, t1 + args.tick * i).sum())
                          for i in range(args.warmup, args.warmup + args.steps))
    el = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    ev = torch.tensor([step_events], dtype=torch.int64, device=cdev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(ev, op=dist.ReduceOp.SUM)
    elapsed = float(el.item())
    total_events = int(ev.item())  # events of all timed steps, all ranks

    kt = np.mean(np.array(kts), axis=0)    # count, scan, map, write_cf, write_walk, offsets (ms)
    nkt = np.mean(np.array(nkts), axis=0)  # join, (transpose +) segments/offsets, node write (ms)
    ms_step = elapsed / args.steps * 1e3

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    if wl == "dispatch":
        print(json.dumps(dispatch_line(args, R, world, elapsed, wake, nkt, build_info,
                                       cpu_dispatch(specs[:args.cpu_sample], t0, args.cpu_threads)
                                       if world == 1 and args.cpu_sample > 0 else None)), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    traffic_src = None
    if pn:
        # per-node CSR bytes: R*32 + nnz*4 + (R+1)*8 + E_n*(8+4) + (N+1)*8
        # per window; the timed interval: k_node_write (its time summed over the
        # windows) -- with --time-order the writer plus the time-order pass
        # behind it (k_ot_*: in the pipelined windows the HIP events around the
        # writer enclose the pass; synchronous windows add the pass's own time)
        nnz, nw = last["nnz"], last["windows"]
        algo_bytes = nw * (R * SPEC_BYTES + nnz * 4 + (R + 1) * 8 + (n_nodes + 1) * 8) + E * 12
        kname, ksec = "k_node_write", nkt[2] / 1e3
        kernels = ["k_node_write"]
        if args.time_order:
            kname = "k_node_write + time-order pass (k_ot_tile, k_ot_merge/mid/big)"
            kernels += ["k_ot_", "k_ts_"]
            if not pn_pipelined:
                ksec += last["order_ms"] / args.steps / 1e3
        hz = f"{H // 3600}h" if H % 3600 == 0 else (f"{H // 86400}d" if H % 86400 == 0 else f"{H}s")
        if wl == "config4":
            metric = f"per-node fire events materialised/sec (config 4: 10M rules × 7d, per-node over 10k nodes)"
            workload = (f"config 4 per node: 10M rules x {hz} (the 1M-rule light-mix block tiled 10x, job-ID "
                        f"order) x 10k nodes (config 3's node model: 500 groups, GroupIDs/NodeIDs/"
                        f"ExcludeNodeIDs), {nw} window(s) of {W}s, {args.zone}, job-ID-range shards over N "
                        f"GPUs; exclude mode {args.exclude_mode}" + (" (job.go:591-630)" if xmode == 0 else ""))
        else:
            metric = f"per-node fire events materialised/sec (config 3: 1M jobs × 10k nodes, {hz})"
            workload = (f"config 3: 1M jobs x 10k nodes (500 groups, GroupIDs/NodeIDs/ExcludeNodeIDs), "
                        f"{'config-2' if wl == 'config3' else 'light'} spec mix, {hz} horizon in "
                        f"{nw} window(s) of {W}s, {args.zone}, per GPU; exclude mode {args.exclude_mode}"
                        + (" (job.go:591-630)" if xmode == 0 else ""))
        tag = {"pernode": "pernode", "config3": "config3", "config4": "config4pn"}[wl] + \
            ("_order" if args.time_order else "")
        if args.zone == "UTC" and xmode == 0:
            traffic_src = pmc_traffic(tag, R, E, kernels, "k_node_write", scale=nw, windows=nw)
    else:
        algo_bytes = R * SPEC_BYTES + E * 8 + (R + 1) * 8   # per rank, per launch
        kname, ksec = "k_write_cf", kt[3] / 1e3
        metric = METRIC
        workload = (f"config 2: 1M mixed cron rules x {H // 3600}h horizon, {args.zone}, per GPU "
                    f"(job-ID-range shards)" if wl == "config2" else
                    f"config 4: 10M rules x 7d horizon, light spec mix, {args.zone}, job-ID-range shards over N GPUs")
        if wl in ("config2", "config4") and args.zone == "UTC" and not args.tick:
            traffic_src = pmc_traffic("" if wl == "config2" else "config4", R, E, ["k_write_cf"], "k_write_cf")
    traffic = traffic_src["bytes"] if traffic_src else None
    achieved = algo_bytes / ksec / 1e9 if ksec > 0 else 0.0

    # the achievable store rate on this box, beside the nominal peak: a
    # vectorized fill of the same output bytes (outside the timed region)
    ceiling = None
    if rank == 0 and wl in ("config2", "pernode") and not args.diagnostic:
        ceiling = store_ceiling(eng, int(E * 12 if pn else E * 8), torch.device("cuda", local), achieved)

    cpu = None
    if world == 1 and args.cpu_sample != 0 and pn:
        a_last = list(range(t0, t1, W))[-1]
        cpu = cpu_baseline_per_node(spec_of, rin, xmode, a_last, min(a_last + W, t1), args.zone)
    if world == 1 and args.cpu_sample != 0 and wl == "config2":
        cpu = cpu_baseline(specs, args.cpu_sample, t0, t1, args.cpu_threads, zone=args.zone)
    if world == 1 and args.cpu_sample != 0 and wl == "config4" and not pn:
        # the 10M-rule set (rule i = base[i % 1M]); a strided sample sized for ~15 s
        cpu = cpu_baseline([spec_of(i) for i in range(R)], args.cpu_sample, t0, t1, args.cpu_threads,
                           zone=args.zone)

    out = {
        "metric": metric,
        "value": total_events / elapsed,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong" if wl == "config4" else "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (seeded spec mix, SURVEY.md §8d; parsed on host, resident in HBM)",
        "config": {
            "workload": workload,
            "rules_per_gpu": R,
            "horizon_s": H,
            "t0": t0,
            "tick_s": args.tick,
            "zone": args.zone,
            "events_per_gpu_step": E,
            "shard": shard_info or {"lo": 0, "hi": R},
            "parallelism": f"dp{world} (job-ID range shards; RCCL allgather of shard totals / per-node counts"
                           + (", through the library's cg_comm)" if lcomm is not None else ")"),
        },
        "hbm_gbps_step": algo_bytes * world / (elapsed / args.steps) / 1e9,
        "steps_mode": ("pipelined (cg_expand_device_async: count/scan of a step overlap the previous "
                       "step's write; one cg_expand_wait at the end of the timed steps)" if pipelined else
                       "synchronous (one call and stream sync per step)") if lean else
                      ("pipelined per-node windows (cg_expand_per_node_rules_device_async: a window's "
                       "expansion and records overlap the previous window's writer, across steps; one "
                       "cg_expand_per_node_wait at the end of the timed steps; "
                       "per-phase times from the synchronous warmup step, node_write from the timed steps)"
                       if pn_pipelined else "synchronous"),
        "kernel_ms": {"count": kt[0], "scan": kt[1], "block_map": kt[2], "write_cf": kt[3],
                      "write_walk": kt[4], "offsets": kt[5],
                      "timing": "write_cf: HIP events around it in the timed steps; the other "
                                "phases from 3 untimed steps with events between all phases"
                                if lean else "HIP events between all phases in the timed steps"},
        "roofline": {
            "bound": "hbm",
            "kernel": kname,
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            # the whole step (every kernel, every window) against the same
            # algorithmic bytes: what a caller of the step gets
            "step_achieved": algo_bytes / (elapsed / args.steps) / 1e9,
            "step_frac": algo_bytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBPS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "timed_interval_s": ksec,
            "algo_bytes_per_launch": algo_bytes,
            "store_ceiling": ceiling,
        },
        "cpu_baseline": cpu,
        "step_wall_ms": {"min": min(step_wall) * 1e3, "p50": float(np.median(step_wall)) * 1e3,
                         "max": max(step_wall) * 1e3},
        "verified": bool(verify and verify["verified_all_ranks"]),
        "verify": verify,
        "library": {"path": os.path.relpath(_cg.LIB_PATH, ROOT), "build_info": build_info},
    }
    if args.diagnostic:
        out["diagnostic"] = {"env": diag_env, "note": "probe/variant run: not a headline"}
    if e2e is not None:
        out["end_to_end_rank0"] = e2e
    if pn:
        # [1]: the (node, rule band) segment records + node offsets of every
        # call, plus the transpose on a call that rebuilds the join
        out["kernel_ms"].update({"rule_node_join": nkt[0], "segments_and_offsets": nkt[1],
                                 "node_write": nkt[2]})
        if args.time_order:  # (time, rule) order of every node's list
            out["kernel_ms"]["time_order"] = last["order_ms"] / args.steps
            out["config"]["per_node_order"] = "(time, rule) within every node (cron.go:64-79 byTime)"
            out["config"]["time_order_by"] = ("cg_node_result_order_by_time after the rule-major writer"
                                              if args.order_pass else
                                              "cg_set_node_order(TIME): the pass inside every (pipelined) "
                                              "per-node call")
        out["config"]["nnz_rule_node_pairs"] = last["nnz"]
        if args.gather_node_csr and world > 1:
            out["config"]["gathered_per_node_csr_on_rank0_events"] = last.get("gathered_events")
        out["config"]["windows"] = last["windows"]
        # the rule->node join + transpose depend only on the uploaded rule set and
        # exclude mode: computed on the first call (warmup), reused afterwards
        out["join_transpose_once_ms"] = {"rule_node_join": last["first_nkt"][0],
                                         "transpose_segments_offsets": last["first_nkt"][1]}
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def rank_launch_cmd(gpus, argv, port):
    """The child that runs N ranks of this same command (one per GPU)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(args):
    """`--gpus N` (N > 1) with no launcher around this process: one child,
    torch.distributed.run with N ranks of this command (node.go:121-141: the
    ranks shard the jobs), started before this process imports torch.cuda,
    loads the library or makes any HIP call (a process that has touched the
    GPU must not start ranks by exec).  Rank 0's JSON line is forwarded to
    stdout, everything else the ranks print to stderr; returns the child's
    exit status.  Inside a launcher (WORLD_SIZE set) returns None, or 2 when
    WORLD_SIZE differs from --gpus."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            log(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}: refusing (one rank per GPU)")
            return 2
        return None
    if args.gpus <= 1:
        return None
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = rank_launch_cmd(args.gpus, sys.argv[1:], port)
    log(f"bench.py: launching {args.gpus} ranks: {' '.join(cmd)}")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    for line in p.stdout:
        if line.lstrip().startswith("{"):
            sys.stdout.write(line)
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    return p.wait()


def gather_check(eng, dist, world, rank, *args, **kw):
    """_gather_check, with a failure reported in the record ({"verified":
    False, "error": ...}) instead of ending the run: the timed line above it
    stays.  The library's calls return the same status on every rank, so the
    ranks fail at the same point and meet at the closing barrier."""
    try:
        return _gather_check(eng, dist, world, rank, *args, **kw)
    except Exception as e:  # noqa: BLE001 -- reported, then the barrier
        log(f"[rank {rank}] gather check failed: {e!r}")
        dist.barrier()
        return {"verified": False, "error": repr(e)[:800]} if rank == 0 else None


def _gather_check(eng, dist, world, rank, backend, loc, zone, t0, dev, cdev, restore_order=0, rules_per_rank=50_000,
                  n_nodes=200, window=600, n_check=24, seed=0x5EED + 91):
    """N > 1, after the timed region: the multi-rank exchange of the per-node
    view, run and verified.  A pernode-shaped job set (`rules_per_rank` jobs
    per rank in job-ID ranges, `n_nodes` nodes, the light spec mix), one
    `window`-second window per rank in (time, rule) order
    (cg_set_node_order(TIME)), gathered on rank 0 with a byte budget of a
    third of the largest node's peer events, so the plan has hundreds of
    chunks and splits nodes: nccl -> the library's communicator
    (cg_comm_gather_node_csr: grouped ncclSend/ncclRecv per chunk,
    k_node_place / k_span_place from the staging buffer, k_merge_ranks over
    the ranks' runs); gloo -> shard.gather_node_csr (the same plan over
    torch.distributed, merged by the library's kernel or numpy).  Rank 0
    checks the offsets and `n_check` seeded nodes' whole lists against the
    oracle (each node filtering every job, node.go:121-141, in its Cron's
    byTime order, cron.go:64-79,220; ties by rule).  Returns the record on
    rank 0 (None elsewhere); every rank returns only after the check."""
    import numpy as np
    import torch
    from cronsun_amd import _lib as cg
    from cronsun_amd import cron, shard, synth
    from cronsun_amd.engine import Comm
    tg = time.perf_counter()
    glob = rules_per_rank * world
    specs = synth.spec_mix(glob, seed=seed, mix=synth.MIX_LIGHT)
    rin = synth.rules_for_nodes(glob, n_nodes=n_nodes, n_groups=20, seed=seed + 1, group_size=(4, 64))
    lo, hi = shard.shard_range(glob, world, rank)
    arr, st = cron.parse_batch(specs[lo:hi], threads=16)
    assert (st == 0).all()
    sp = eng.upload_c(arr, hi - lo)
    drules = eng.upload_rules(rin.slice_rules(lo, hi))
    eng.set_node_order(cg.NODE_ORDER_TIME)
    try:
        En, _ = eng.expand_per_node_rules_device(sp, loc, t0, t0 + window, drules, cg.EXCLUDE_NONE)
    finally:
        eng.set_node_order(restore_order)
    n_off, n_time, n_rule = eng.node_result_tensors(n_nodes)
    cnt = (n_off[1:] - n_off[:-1]).to(cdev)
    allc = torch.zeros(world * n_nodes, dtype=torch.int64, device=cdev)
    dist.all_gather_into_tensor(allc, cnt.contiguous())
    allc = allc.view(world, n_nodes).cpu().numpy()
    peer = allc.sum(axis=0) - allc[0]
    budget = 12 * max(2 * world, int(peer.max()) // 3)
    plan = shard.node_gather_plan(allc, 0, budget)
    total = int(allc.sum())
    tx = time.perf_counter()
    out = None
    if backend == "nccl":
        uid = [Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = Comm(eng, world, rank, uid[0])
        try:
            if rank == 0:
                o = torch.empty(n_nodes + 1, dtype=torch.int64, device=dev)
                t = torch.full((total,), -1, dtype=torch.int64, device=dev)
                r = torch.full((total,), -1, dtype=torch.int32, device=dev)
                torch.cuda.synchronize(dev)
                n = comm.gather_node_csr(0, lo, budget, o.data_ptr(), t.data_ptr(), r.data_ptr(), total)
                out = (o.cpu().numpy(), t.cpu().numpy(), r.cpu().numpy(), n)
            else:
                comm.gather_node_csr(0, lo, budget)
        finally:
            comm.free()
        how = "cg_comm_gather_node_csr (the library's RCCL communicator)"
    else:
        g = shard.gather_node_csr(n_off.to(cdev), n_time.to(cdev), n_rule.to(cdev), lo, dist, engine=eng,
                                  budget_bytes=budget, order="time")
        if rank == 0:
            out = (g[0].cpu().numpy(), g[1].cpu().numpy(), g[2].cpu().numpy(), int(g[1].numel()))
        how = "shard.gather_node_csr over torch.distributed (gloo)"
    t_gather = time.perf_counter() - tx
    sp.free()
    drules.free()
    res = None
    if rank == 0:
        O = _oracle()
        off, gt, gr, n = out
        nodes = np.sort(np.random.default_rng(seed + 2).choice(n_nodes, n_check, replace=False))
        roff, rules = O.node_rules(rin, 0, nodes, threads=host_cpus()[0])
        union = np.unique(rules)
        eo, et = O.expand_batch(_oracle_scheds(O, [specs[int(i)] for i in union]), t0, t0 + window,
                                O.Loc(zone), threads=host_cpus()[0])
        bad, ev = 0, 0
        for k, nd in enumerate(nodes):
            pos = np.searchsorted(union, rules[roff[k]:roff[k + 1]])
            exp_t, exp_p = O.node_list(eo, et, pos)
            o = np.lexsort((exp_p, exp_t))  # (time, rule): pos ascends with the global rule
            exp_t, exp_r = exp_t[o], union[exp_p[o]]
            a, b = int(off[nd]), int(off[nd + 1])
            ev += len(exp_t)
            bad += not (np.array_equal(gt[a:b], exp_t) and np.array_equal(gr[a:b], exp_r))
        exp_off = np.concatenate([[0], np.cumsum(allc.sum(axis=0))])
        offs_ok = bool(np.array_equal(off, exp_off) and n == total)
        split = sum(1 for c in plan if c[3] > 1)
        res = {"verified": bad == 0 and offs_ok, "via": how,
               "shape": f"{glob} jobs ({rules_per_rank} per rank) x {n_nodes} nodes, light mix, {window}-s window, "
                        f"(time, rule) order per node",
               "events": total, "budget_bytes": budget, "chunks": len(plan), "split_node_chunks": split,
               "nodes_checked": int(len(nodes)), "events_checked": int(ev), "mismatched_nodes": int(bad),
               "offsets_consistent": offs_ok, "gather_s": t_gather, "seconds": time.perf_counter() - tg}
    dist.barrier()
    return res


def dispatch_line(args, R, world, elapsed, wake, nkt, build_info, cpu):
    import numpy as np
    wall = np.array(wake["wall"] or [0.0])
    due = wake["due"] / max(wake["wakes"], 1)
    # k_dispatch_scan per launch: read Next of every entry (8 B) and write the
    # due bitmap (1 bit); the advance pass then reads the due entries' spec
    # (32 B) and Next (8 B) and writes Prev/Next (16 B)
    algo = R * 8 + R / 8
    fire_s = nkt[0] / 1e3
    achieved = algo / fire_s / 1e9 if fire_s > 0 else 0.0
    return {
        "metric": "dispatcher entries scanned/sec (Cron.run wake over 10M entries)",
        "value": R * world * args.steps / elapsed,
        "unit": "entries/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (config-2 spec mix, seeded; parsed on host, resident in HBM)",
        "config": {"workload": "dispatch: Cron.run entry table of 10M config-2 rules per GPU "
                               "(the 1M-rule set tiled), on-time wakes from 2026-01-01 UTC",
                   "entries_per_gpu": R, "zone": "UTC", "mean_due_per_wake": due,
                   "parallelism": f"dp{world} (independent entry tables)"},
        "wakes_per_s": args.steps / elapsed,
        "timed_split_s": {"loop": wake["loop_s"], "final_sync_barrier": wake["tail_s"],
                          "fire_calls": float(wall.sum())},
        "wake_wall_us": {q: float(np.percentile(wall, p)) * 1e6 for q, p in
                         (("p50", 50), ("p90", 90), ("p99", 99), ("max", 100))},
        "kernel_ms": {"scan": nkt[0], "compact": nkt[1], "advance": nkt[2],
                      "wake_total": float(sum(nkt))},
        "roofline": {"bound": "hbm", "kernel": "k_dispatch_scan", "achieved": achieved,
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS,
                     "traffic": None, "algo_bytes_per_launch": algo},
        "cpu_baseline": cpu,
        "verified": None,
        "verify": "dispatcher wakes are checked wake by wake against the oracle in "
                  "tests/test_gpu_dispatch.py, not in the bench",
        "library": {"build_info": build_info},
    }


def parse_line(args):
    """the batch parser (cg_parse_batch: parser.go:78-377
    restated in C++, Go's error texts) over 10M spec strings of the config-2
    mix on the host's CPUs; beside it the oracle's parser (the same semantics,
    one spec per call) on one thread."""
    import ctypes as C
    import numpy as np
    from cronsun_amd import _lib, synth
    n_total = args.rules or 10_000_000
    base = synth.spec_mix(1_000_000, seed=0x5EED)
    enc = [s.encode() for s in base]
    reps = (n_total + len(enc) - 1) // len(enc)
    enc = (enc * reps)[:n_total]
    bufs = (C.c_char_p * n_total)(*enc)
    lens = np.array([len(b) for b in enc], dtype=np.uint64)
    out = (_lib.cg_schedule * n_total)()
    status = np.zeros(n_total, dtype=np.int32)
    threads, cpuinfo = host_cpus()
    times = []
    for _ in range(max(1, args.warmup) + max(1, args.steps)):
        t = time.perf_counter()
        _lib.check(_lib.lib().cg_parse_batch(_lib.PARSE_DEFAULT, C.cast(bufs, C.c_void_p), lens.ctypes.data,
                                             n_total, C.cast(out, C.c_void_p), status.ctypes.data, threads))
        times.append(time.perf_counter() - t)
    assert (status == 0).all()
    dt = float(np.median(times[max(1, args.warmup):]))
    O = _oracle()
    sample = base[:200_000]
    t = time.perf_counter()
    for s in sample:
        O.parse(s)
    dto = time.perf_counter() - t
    return {"metric": "cron specs parsed/sec (host batch parser, 10M config-2 specs)",
            "value": n_total / dt, "unit": "specs/s", "n_gpus": 0, "steps": max(1, args.steps),
            "warmup": max(1, args.warmup), "ms_per_step": dt * 1e3, "higher_is_better": True,
            "scaling": "none", "vs_baseline": None, "dtype": "bytes", "data": "synthetic config-2 mix",
            "config": {"workload": "parse: 10M spec strings (the 1M config-2 mix repeated), "
                                   "cg_parse_batch, default options (parser.go:171-183)",
                       "threads": threads, **cpuinfo},
            "cpu_baseline": {"value": len(sample) / dto, "unit": "specs/s", "cores": 1, "kind": "port",
                             "sample": f"the oracle's parser over the first {len(sample)} specs, one "
                                       f"call per spec through ctypes ({dto:.2f} s)"}}


def host_cpus():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU
    quota when one is set (a GPU box's share of a larger host)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except Exception:
        pass
    return (min(aff, quota) if quota else aff), {"affinity_cpus": aff, "cgroup_quota_cpus": quota}


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    return O


def _oracle_scheds(O, specs):
    memo, out = {}, []
    for s in specs:
        if s not in memo:
            sc, err = O.parse(s)  # the oracle's own parser (parser.go restated)
            if err is not None:
                raise RuntimeError(f"oracle rejects {s!r}: {err}")
            memo[s] = sc
        out.append(memo[s])
    return O.sched_array(out)


def verify_rule_major(eng, spec_of, R, t0, t1, E, sample, seed, zone="UTC"):
    """The last timed step's rule-major CSR against the oracle's Next loop on
    a seeded sample of rules (checker only; outside the timed region)."""
    import numpy as np
    from cronsun_amd._lib import check, lib
    O = _oracle()
    off = np.empty(R + 1, dtype=np.int64)
    check(lib().cg_result_copy_offsets(eng._h, off.ctypes.data))
    idx = np.sort(np.random.default_rng(seed).choice(R, min(sample, R), replace=False))
    eo, et = O.expand_batch(_oracle_scheds(O, [spec_of(int(i)) for i in idx]), t0, t1, O.Loc(zone),
                            threads=host_cpus()[0])
    bad = 0
    for k, i in enumerate(idx):
        got = eng.copy_times(off[i], off[i + 1] - off[i])
        bad += not np.array_equal(got, et[eo[k]:eo[k + 1]])
    mono = bool(off[0] == 0 and off[-1] == E and (np.diff(off) >= 0).all())
    return {"verified": bad == 0 and mono, "kind": "rule-major CSR vs oracle Next loop",
            "rules_checked": int(len(idx)), "events_checked": int(eo[-1]),
            "mismatched_rules": int(bad), "offsets_consistent": mono}


def verify_per_node(eng, spec_of, rin, mode, a, b, En, n_nodes_sample, seed, zone="UTC", time_order=False):
    """The last timed window's per-node lists against each sampled node's own
    filter over every rule (node.go:121-158 -> Job.Cmds) composed with the
    oracle's Next loop (checker only; outside the timed region)."""
    import numpy as np
    from cronsun_amd._lib import check, lib
    O = _oracle()
    threads = host_cpus()[0]
    node_off = np.empty(rin.n_nodes + 1, dtype=np.int64)
    check(lib().cg_node_result_copy(eng._h, node_off.ctypes.data, None, None, 0))
    nodes = np.sort(np.random.default_rng(seed).choice(rin.n_nodes, n_nodes_sample, replace=False))
    roff, rules = O.node_rules(rin, mode, nodes, threads=threads)
    union = np.unique(rules)
    eo, et = O.expand_batch(_oracle_scheds(O, [spec_of(int(r)) for r in union]), a, b, O.Loc(zone),
                            threads=threads)
    bad, ev = 0, 0
    for k, n in enumerate(nodes):
        pos = np.searchsorted(union, rules[roff[k]:roff[k + 1]])
        exp_t, exp_p = O.node_list(eo, et, pos)
        if time_order:  # (time, rule) order: pos ascends with the rule index
            o = np.lexsort((exp_p, exp_t))
            exp_t, exp_p = exp_t[o], exp_p[o]
        got_t, got_r = eng.node_copy_range(node_off[n], node_off[n + 1] - node_off[n])
        ev += len(exp_t)
        bad += not (np.array_equal(got_t, exp_t) and np.array_equal(got_r, union[exp_p]))
    mono = bool(node_off[0] == 0 and node_off[-1] == En and (np.diff(node_off) >= 0).all())
    return {"verified": bad == 0 and mono, "kind": "per-node lists of the last window vs oracle",
            "nodes_checked": int(len(nodes)), "events_checked": int(ev),
            "mismatched_nodes": int(bad), "offsets_consistent": mono}


def verify_window_checksums(eng, spec_of, rin, mode, t0, t1, W, ck, zone="UTC", time_order=False):
    """Every timed step's seeded window: the device checksums of the sample
    nodes' lists (cg_node_checksum_enqueue, taken in the timed region right
    behind that window's writer) against the same checksums of the oracle's
    lists (the nodes' own filter over every rule composed with the Next loop
    started at the window's start)."""
    import numpy as np
    O = _oracle()
    threads = host_cpus()[0]
    nodes = ck["nodes_np"]
    roff, rules = O.node_rules(rin, mode, nodes, threads=threads)
    union = np.unique(rules)
    osch = _oracle_scheds(O, [spec_of(int(r)) for r in union])
    loc = O.Loc(zone)
    got = ck["out"].cpu().numpy().view(np.uint64)
    wins = list(range(t0, t1, W))
    exp = {}  # window -> per node (times, rules)
    bad = 0
    for s, wi in enumerate(ck["win"]):
        wi = int(wi)
        if wi not in exp:
            a, b = wins[wi], min(wins[wi] + W, t1)
            eo, et = O.expand_batch(osch, a, b, loc, threads=threads)
            exp[wi] = []
            for k in range(len(nodes)):
                pos = np.searchsorted(union, rules[roff[k]:roff[k + 1]])
                exp_t, exp_p = O.node_list(eo, et, pos)
                exp_r = union[exp_p]
                if time_order:
                    o = np.argsort(exp_t, kind="stable")  # rule-major input: stable by time = (time, rule)
                    exp_t, exp_r = exp_t[o], exp_r[o]
                exp[wi].append(eng.node_list_checksum(exp_t, exp_r))
        for k in range(len(nodes)):
            ct, cr = exp[wi][k]
            bad += not (int(got[s, 2 * k]) == ct and int(got[s, 2 * k + 1]) == cr)
    return {"verified": bad == 0, "kind": "every timed step: a seeded window's lists of 8 sample nodes, "
            "device checksums taken behind its writer vs the oracle's", "steps": int(len(ck["win"])),
            "windows": [int(x) for x in ck["win"]], "nodes": [int(x) for x in nodes],
            "mismatches": int(bad)}


def cpu_dispatch(specs, t0, threads=0):
    """The reference's wake (sort.Sort(byTime) + Next for the due prefix,
    cron.go:220-244) as the oracle's C port, on a bounded sample, on all of
    this host's CPUs: the sample is split into one Cron per thread (the
    reference runs one single-goroutine Cron per node process; here each
    thread is such a Cron over its share of the entries, all waking on the
    same schedule), and the time of one steady-state wake of all of them
    (after the start wake has sorted every table) is reported."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    from concurrent.futures import ThreadPoolExecutor
    import oracle_lib as O
    avail, cpuinfo = host_cpus()
    T = max(1, min(threads or avail, len(specs)))
    memo = {}
    scheds = []
    for sp in specs:
        if sp not in memo:
            memo[sp] = O.parse(sp)[0]
        scheds.append(memo[sp])
    loc = O.Loc("UTC")
    L = O.lib()
    shards = []
    for k in range(T):
        part = scheds[k * len(scheds) // T:(k + 1) * len(scheds) // T]
        arr = (O.OrEntry * len(part))()
        for i, sc in enumerate(part):
            arr[i].s = C.pointer(sc)
            arr[i].id = i
        shards.append((arr, len(part), (C.c_int32 * max(len(part), 1))()))
    for arr, n, _ in shards:
        L.or_cron_start(arr, n, t0, loc.h)

    def wake(sh):  # ctypes releases the GIL for the C call
        arr, n, ids = sh
        e = L.or_cron_effective(arr, n)
        L.or_cron_fire(arr, n, e, e, loc.h, ids)

    with ThreadPoolExecutor(T) as ex:
        list(ex.map(wake, shards))  # the first wake after the start
        ts = time.perf_counter()
        wakes = 0
        while time.perf_counter() - ts < 5.0 and wakes < 50:
            list(ex.map(wake, shards))
            wakes += 1
        dt = (time.perf_counter() - ts) / wakes
    return {"value": len(scheds) / dt, "unit": "entries/s", "cores": T, "kind": "port",
            "sample": f"{len(scheds)} entries of the same mix in {T} Cron tables (one per thread), {wakes} "
                      f"steady-state wakes ({dt * 1e3:.1f} ms per wake: qsort by Next + Next for the due "
                      f"prefix, every table)", **cpuinfo}


def cpu_baseline_per_node(spec_of, rin, mode, a, b, zone, n_nodes=24, seed=0x5EED + 55):
    """The reference's per-node work on the host (oracle port, all host CPUs):
    every node filters all jobs (node.go:121-158 -> Job.Cmds) and runs the
    Next loop of its rules over the window, then lists its (time, rule)
    events -- timed on a seeded sample of nodes, events/s over the sample."""
    import numpy as np
    O = _oracle()
    threads, cpuinfo = host_cpus()
    loc = O.Loc(zone)
    nodes = np.sort(np.random.default_rng(seed).choice(rin.n_nodes, n_nodes, replace=False))
    ts = time.perf_counter()
    roff, rules = O.node_rules(rin, mode, nodes, threads=threads)
    t_filter = time.perf_counter() - ts
    events = 0
    for k in range(len(nodes)):
        rs = rules[roff[k]:roff[k + 1]]
        eo, et = O.expand_batch(_oracle_scheds(O, [spec_of(int(r)) for r in rs]), a, b, loc, threads=threads)
        O.node_list(eo, et, np.arange(len(rs)))
        events += int(eo[-1])
    dt = time.perf_counter() - ts
    return {"value": events / dt, "unit": "node events/s", "cores": threads, "kind": "port",
            "sample": f"{len(nodes)} nodes of {rin.n_nodes}: each filters all {rin.n_rules} rules "
                      f"({t_filter:.2f} s for the sample) then expands its rules over ({a}, {b}] and lists "
                      f"its events ({events} node events, {dt:.2f} s; parse of the rules' specs included)",
            **cpuinfo}


def cpu_baseline(specs, sample, t0, t1, threads, zone="UTC"):
    """The oracle's literal Next loop (reference semantics, port of
    spec.go:55-158 + Go time) on this host's CPUs: one pass of
    `t = Next(t)` until > T1 per rule, parallel over rules (the Go baseline's
    goroutine worker pool).  sample < 0: a strided calibration
    sample first, then the whole workload if it fits ~30 s, else a strided
    sample sized for ~15 s; sample > 0: that many rules, strided."""
    O = _oracle()
    avail, cpuinfo = host_cpus()
    threads = threads or avail
    loc = O.Loc(zone)

    def timed(sub):
        tp = time.perf_counter()
        arr = _oracle_scheds(O, sub)
        parse_s = time.perf_counter() - tp
        ts = time.perf_counter()
        off, _ = O.expand_batch(arr, t0, t1, loc, threads=threads, with_times=False)
        return int(off[-1]), time.perf_counter() - ts, parse_s

    n = len(specs)
    if sample < 0:
        stride = max(1, n // 20_000)
        ev, dt, _ = timed(specs[::stride])
        est = dt * stride
        if est <= 30.0:
            sample = n
        else:
            sample = max(20_000, int(n * 15.0 / est))
    stride = max(1, n // sample)
    sub = specs[::stride][:sample]
    ev, dt, parse_s = timed(sub)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    what = ("the whole workload" if len(sub) == n else
            f"every {stride}th rule ({len(sub)} of {n})")
    return {"value": ev / dt, "unit": "events/s", "cores": threads, "kind": "port",
            "sample": f"{what} x {t1 - t0}s horizon, {zone} ({ev} events, {dt:.2f}s for one pass of "
                      f"the Next loop on {threads} threads; parse excluded, +{parse_s:.2f}s parse)",
            "value_incl_parse": ev / (dt + parse_s), "cpu_model": cpu_model, **cpuinfo,
            "go_toolchain": "absent on the box image (oracle C port timed instead)"}


if __name__ == "__main__":
    main()
