"""Multi-GPU sharding of the expansion.

Rules are independent, so ranks take contiguous job-ID ranges and expand them
with no data-path collective.  The only exchanges are small:

  global_offsets   all-gather of per-rank event totals -> each rank's base
                   offset in the global rule-major CSR
  event_balanced_range
                   the cheap count pass: each rank counts the fires of a
                   provisional equal slice, the per-block sums are
                   all-gathered, and every rank cuts the job-ID order into
                   ranges of equal estimated events (block granularity)
  node_offsets     all-gather of per-node event counts (N int64 per rank) ->
                   offset[g][n] = node_base[n] + sum_{g' < g} count[g'][n], so
                   each node's global list keeps job-ID order across ranks

  gather_csr       the optional second collective: every rank's slice of the
                   rule-major CSR to rank 0 with grouped point-to-point
                   send/recv (variable sizes; xGMI: one link per peer)
  gather_node_csr  the same for the per-node CSR (north_star's "gather the
                   final per-node CSR"): every node's global list is the
                   ranks' slices of it in job-ID order, as one process walking
                   all jobs builds it (node/node.go:121-158 -> Job.Cmds), or
                   for time-ordered lists those slices merged by (time, rule)
                   (merge_rank_runs; the node's byTime order); in
                   chunks of node ranges under a byte budget, so the
                   destination stages at most the budget beside its output
                   (the library's cg_comm_gather_node_csr does the same over
                   RCCL behind the C-ABI)

Works with torch.distributed over RCCL ("nccl", one process per MI355X) and
over gloo on CPU (tests).
"""
import numpy as np


def shard_range(n_rules, world, rank, weights=None):
    """[lo, hi) job-ID range of `rank`.  With `weights` (e.g. estimated events
    per rule) the split balances the weight instead of the rule count."""
    if world <= 1:
        return 0, n_rules
    if weights is None:
        lo = n_rules * rank // world
        hi = n_rules * (rank + 1) // world
        return lo, hi
    w = np.asarray(weights, dtype=np.float64)
    c = np.concatenate([[0.0], np.cumsum(w)])
    total = c[-1]
    def cut(target):  # the prefix boundary nearest to the target weight
        k = int(np.searchsorted(c, target, side="left"))
        if k > 0 and (k > n_rules or target - c[k - 1] <= c[k] - target):
            return k - 1
        return k
    cuts = [0] + [cut(total * k / world) for k in range(1, world)] + [n_rules]
    cuts = np.maximum.accumulate(np.clip(cuts, 0, n_rules))
    return int(cuts[rank]), int(cuts[rank + 1])


def provisional_blocks(n_rules, world, rank, block):
    """[b0, b1) block range of an equal split in blocks of `block` rules."""
    nb = (n_rules + block - 1) // block
    return nb * rank // world, nb * (rank + 1) // world


def event_balanced_range(n_rules, count_fn, dist, block=4096, device=None):
    """This rank's [lo, hi) job-ID range with balanced estimated events.

    count_fn(lo, hi) -> per-rule event counts of rules [lo, hi) (e.g.
    Engine.count over the rank's provisional slice).  One all-gather of
    ceil(blocks / world) int64 per rank; the cut is made at block
    granularity, so every rank computes the same cuts and job-ID order is
    kept.  Returns (lo, hi, global block weights)."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    nb = (n_rules + block - 1) // block
    b0, b1 = provisional_blocks(n_rules, world, rank, block)
    lo, hi = b0 * block, min(b1 * block, n_rules)
    counts = np.asarray(count_fn(lo, hi), dtype=np.int64) if hi > lo else np.zeros(0, np.int64)
    mine = np.zeros(b1 - b0, dtype=np.int64)
    if hi > lo:
        mine = np.add.reduceat(counts, np.arange(0, hi - lo, block))
    width = (nb + world - 1) // world + 1
    buf = torch.zeros(width, dtype=torch.int64, device=device)
    buf[:len(mine)] = torch.from_numpy(mine).to(buf.device)
    allw = torch.zeros(world * width, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(allw, buf)
    allw = allw.cpu().numpy().reshape(world, width)
    weights = np.concatenate([allw[g, :provisional_blocks(n_rules, world, g, block)[1] -
                                   provisional_blocks(n_rules, world, g, block)[0]]
                              for g in range(world)])
    c0, c1 = shard_range(nb, world, rank, weights=weights.astype(np.float64) + 1e-9)
    return c0 * block, min(c1 * block, n_rules), weights


def global_offsets(local_total, dist, device=None):
    """-> (base offset of this rank in the global CSR, global total,
    per-rank totals) via one all-gather."""
    import torch
    world = dist.get_world_size()
    mine = torch.tensor([int(local_total)], dtype=torch.int64, device=device)
    out = torch.zeros(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(out, mine)
    tot = out.cpu().numpy()
    r = dist.get_rank()
    return int(tot[:r].sum()), int(tot.sum()), tot


def node_offsets(local_counts, dist):
    """local_counts: torch int64 tensor [N] (this rank's per-node event counts,
    on the collective's device).  Returns (offset[N] of this rank's slice of
    every node's global list, node_base[N+1] global node CSR offsets)."""
    import torch
    world = dist.get_world_size()
    r = dist.get_rank()
    N = local_counts.numel()
    allc = torch.zeros(world * N, dtype=torch.int64, device=local_counts.device)
    dist.all_gather_into_tensor(allc, local_counts.contiguous())
    allc = allc.view(world, N)
    per_node_total = allc.sum(dim=0)
    node_base = torch.zeros(N + 1, dtype=torch.int64, device=local_counts.device)
    node_base[1:] = torch.cumsum(per_node_total, dim=0)
    before = allc[:r].sum(dim=0) if r > 0 else torch.zeros(N, dtype=torch.int64, device=local_counts.device)
    return node_base[:-1] + before, node_base


def gather_csr(local_offsets, local_times, dist, dst=0):
    """Gather the job-ID-ordered rule-major CSR on rank `dst`.

    local_offsets: int64 tensor [R_local + 1] (starting at 0), local_times:
    int64 tensor [E_local], on the collective's device.  Returns (offsets
    [R + 1], times [E]) on `dst` (None elsewhere).  Sizes are exchanged with
    one all-gather; the payload moves with batched isend/irecv, each peer
    straight into its slice of the destination buffers."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = local_times.device
    sizes = torch.tensor([local_offsets.numel() - 1, local_times.numel()], dtype=torch.int64, device=dev)
    alls = torch.zeros(world * 2, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(alls, sizes)
    alls = alls.view(world, 2).cpu().numpy()
    if rank != dst:
        ops = [dist.P2POp(dist.isend, local_offsets.contiguous(), dst),
               dist.P2POp(dist.isend, local_times.contiguous(), dst)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        return None
    R, E = int(alls[:, 0].sum()), int(alls[:, 1].sum())
    offsets = torch.zeros(R + 1, dtype=torch.int64, device=dev)
    times = torch.empty(E, dtype=torch.int64, device=dev)
    rbase = np.concatenate([[0], np.cumsum(alls[:, 0])])
    ebase = np.concatenate([[0], np.cumsum(alls[:, 1])])
    recv_off, ops = {}, []
    for g in range(world):
        if g == dst:
            continue
        recv_off[g] = torch.empty(int(alls[g, 0]) + 1, dtype=torch.int64, device=dev)
        ops.append(dist.P2POp(dist.irecv, recv_off[g], g))
        ops.append(dist.P2POp(dist.irecv, times[int(ebase[g]):int(ebase[g + 1])], g))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for g in range(world):
        lo = int(rbase[g])
        part = local_offsets if g == dst else recv_off[g]
        if g == dst:
            times[int(ebase[g]):int(ebase[g + 1])] = local_times
        offsets[lo:lo + int(alls[g, 0]) + 1] = part + int(ebase[g])
    return offsets, times


def node_slice_starts(allc, rank):
    """Per-node destinations of rank `rank`'s slices in the gathered per-node
    CSR: node_base[n] + sum_{g' < rank} count[g'][n] (allc: [world, N]
    all-gathered counts).  Returns (starts [N], node_base [N + 1])."""
    import torch
    per_node = allc.sum(dim=0)
    node_base = torch.zeros(allc.shape[1] + 1, dtype=torch.int64, device=allc.device)
    node_base[1:] = torch.cumsum(per_node, dim=0)
    before = allc[:rank].sum(dim=0) if rank > 0 else torch.zeros_like(per_node)
    return node_base[:-1] + before, node_base


def place_node_slice(node_off, time, rule, rule_add, starts, out_time, out_rule, engine=None):
    """Copy one rank's per-node slice (node_off [N+1] from 0, time, rule) to
    out_time / out_rule at starts[n] per node, rules + rule_add.  Device
    tensors go through the library's kernel (cg_node_csr_place); host tensors
    (gloo runs on CPU) are copied per node."""
    import torch
    N = node_off.numel() - 1
    if time.is_cuda:
        if engine is None:
            if (time.device.index or 0) != 0:
                raise ValueError("place_node_slice: pass the Engine of the tensors' device")
            from .engine import default_engine
            engine = default_engine()
        elif engine.device != (time.device.index or 0):
            raise ValueError(f"place_node_slice: engine on device {engine.device}, tensors on {time.device}")
        torch.cuda.synchronize(time.device)  # the library runs on its own stream
        engine.node_csr_place(N, node_off.data_ptr(), time.data_ptr(), rule.data_ptr(), int(rule_add),
                              starts.contiguous().data_ptr(), out_time.data_ptr(), out_rule.data_ptr())
        return
    off = node_off.numpy()
    st = starts.numpy()
    t, r = time.numpy(), rule.numpy()
    ot, orl = out_time.numpy(), out_rule.numpy()
    for n in range(N):
        a, b = int(off[n]), int(off[n + 1])
        if b > a:
            ot[st[n]:st[n] + b - a] = t[a:b]
            orl[st[n]:st[n] + b - a] = r[a:b] + rule_add


def node_gather_plan(allc, dst, budget_bytes):
    """The chunks of the per-node CSR gather, the same on every rank (the
    library's cg_comm_gather_node_csr plans identically, cg_comm.cpp): whole
    node ranges [n0, n1) whose peer events (every rank but `dst`, 12 B each)
    fit the budget, and a node with more peer events than that in k parts
    (part j of rank g: its events [c*j//k, c*(j+1)//k) of that node).
    allc: numpy int64 [world, N] per-node counts.  Returns [(n0, n1, j, k)]."""
    allc = np.asarray(allc, dtype=np.int64)
    world, N = allc.shape
    cap_ev = int(budget_bytes) // 12
    if world > 1 and cap_ev < 2 * world:
        raise ValueError("gather budget below 24 bytes per rank")
    P = allc.sum(axis=0) - allc[dst]
    out = []
    n = 0
    while n < N:
        if P[n] > cap_ev:
            per = cap_ev - (world - 1)
            k = (int(P[n]) + per - 1) // per
            out += [(n, n + 1, j, k) for j in range(k)]
            n += 1
            continue
        n0, acc = n, 0
        while n < N and P[n] <= cap_ev and acc + P[n] <= cap_ev:
            acc += int(P[n])
            n += 1
        if acc > 0:
            out.append((n0, n, 0, 1))
    return out


def _piece(off_g, cnt_g, chunk):
    """Rank g's events [lo, hi) of its own CSR in a chunk."""
    n0, n1, j, k = chunk
    a = int(off_g[n0])
    if k == 1:
        return a, int(off_g[n1])
    c = int(cnt_g[n0])
    return a + c * j // k, a + c * (j + 1) // k


DEFAULT_GATHER_BUDGET = 1 << 31  # bytes of peer events staged on dst per chunk


def merge_rank_runs(run_bounds, out_time, out_rule, engine=None, budget_bytes=DEFAULT_GATHER_BUDGET):
    """Merge every node's rank slices of a gathered per-node CSR into (time,
    rule) order, in place (the byTime order of the node's Cron,
    cron.go:64-79,220, over every job).  run_bounds: numpy int64 [N, world+1],
    run g of node n = [rb[n, g], rb[n, g+1]), each run already in (time, rule)
    order and rank g's rules below rank g+1's, so a stable sort by time per
    node is the (time, rule) order.  Device tensors go through the library
    (cg_node_csr_merge_ranks), host tensors through numpy."""
    import torch
    rb = np.asarray(run_bounds, dtype=np.int64)
    N, w1 = rb.shape
    if w1 <= 2 or N == 0:
        return
    if out_time.is_cuda:
        if engine is None:
            if (out_time.device.index or 0) != 0:
                raise ValueError("merge_rank_runs: pass the Engine of the tensors' device")
            from .engine import default_engine
            engine = default_engine()
        elif engine.device != (out_time.device.index or 0):
            raise ValueError(f"merge_rank_runs: engine on device {engine.device}, tensors on {out_time.device}")
        torch.cuda.synchronize(out_time.device)  # the library runs on its own stream
        engine.node_csr_merge_ranks(N, w1 - 1, rb, out_time.data_ptr(), out_rule.data_ptr(), budget_bytes)
        return
    t, r = out_time.numpy(), out_rule.numpy()
    for n in range(N):
        a, b = int(rb[n, 0]), int(rb[n, -1])
        if b - a > 1:
            o = np.argsort(t[a:b], kind="stable")
            t[a:b], r[a:b] = t[a:b][o], r[a:b][o]


def gather_node_csr(local_node_off, local_time, local_rule, rule_base, dist, dst=0, engine=None,
                    budget_bytes=DEFAULT_GATHER_BUDGET, *, order):
    """Gather the per-node (time, rule) CSR of job-ID-range shards on rank `dst`.

    local_node_off: int64 tensor [N+1] (this rank's node offsets, from 0);
    local_time int64 [E_g] and local_rule int32 [E_g] (rule indices local to
    the rank's range, which starts at global rule `rule_base`), all on the
    collective's device.  `order` (required) is the order of every rank's
    lists: "rule" (rule-major, the default per-node order: the gathered list
    is the ranks' slices in job-ID order) or "time" ((time, rule) order,
    cg_set_node_order(TIME): the slices are then merged per node by (time,
    global rule) -- concatenating them would not be in time order).  Returns
    (node_off [N+1], time [E], rule [E], global rule indices) on `dst`, None
    elsewhere.

    Sizes: one all-gather of the per-node counts (N int64 per rank, the
    collective node_offsets uses).  Payload: in chunks of node ranges
    (node_gather_plan) whose peer events stay within budget_bytes, so dst
    stages at most that much beside its output: per chunk every peer's piece
    (one contiguous range of its CSR) moves with batched isend/irecv into a
    staging buffer, then each piece is placed at node_base[n] +
    sum_{g' < g} count[g'][n] by the library's placement kernel
    (cg_node_csr_place; rule indices made global there).  dst's own slice is
    placed straight from its buffers."""
    import torch
    if order not in ("rule", "time"):
        raise ValueError(f"gather_node_csr: order must be 'rule' or 'time', not {order!r}")
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = local_time.device
    N = local_node_off.numel() - 1
    counts = (local_node_off[1:] - local_node_off[:-1]).to(torch.int64).contiguous()
    allc = torch.zeros(world * N, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allc, counts)
    allc = allc.view(world, N)
    allc_h = allc.cpu().numpy()
    # every rank's range base (the placement makes rule indices global)
    base_t = torch.tensor([int(rule_base)], dtype=torch.int64, device=dev)
    bases = torch.zeros(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(bases, base_t)
    bases = bases.cpu().numpy()
    if order == "time":
        # the merge breaks time ties by rank: (time, global rule) order only
        # when the job-ID ranges of the ranks holding events ascend with the
        # rank (every rank sees the same bases and totals, so all raise)
        held = bases[allc_h.sum(axis=1) > 0]
        if len(held) > 1 and not (np.diff(held) > 0).all():
            raise ValueError("gather_node_csr: rule_base does not ascend with the rank "
                             "(time-ordered slices merge by rank)")
    offs = np.zeros((world, N + 1), dtype=np.int64)
    offs[:, 1:] = np.cumsum(allc_h, axis=1)
    plan = node_gather_plan(allc_h, dst, budget_bytes)
    lt, lr = local_time.contiguous(), local_rule.contiguous()
    if rank != dst:
        for ch in plan:
            lo, hi = _piece(offs[rank], allc_h[rank], ch)
            if hi > lo:
                ops = [dist.P2POp(dist.isend, lt[lo:hi], dst), dist.P2POp(dist.isend, lr[lo:hi], dst)]
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
        return None
    E = int(offs[:, -1].sum())
    out_time = torch.empty(E, dtype=torch.int64, device=dev)
    out_rule = torch.empty(E, dtype=torch.int32, device=dev)
    starts = [node_slice_starts(allc, g)[0] for g in range(world)]
    node_base = node_slice_starts(allc, dst)[1]
    starts_h = [x.cpu().numpy() for x in starts]
    if int(offs[dst, -1]) > 0:  # dst's own slice
        place_node_slice(local_node_off, lt, lr, int(bases[dst]), starts[dst], out_time, out_rule, engine)
    pieces = [[_piece(offs[g], allc_h[g], ch) if g != dst else (0, 0) for g in range(world)] for ch in plan]
    stage_n = max([sum(hi - lo for lo, hi in p) for p in pieces] or [0])
    stage_t = torch.empty(max(stage_n, 1), dtype=torch.int64, device=dev)
    stage_r = torch.empty(max(stage_n, 1), dtype=torch.int32, device=dev)
    for ch, pc in zip(plan, pieces):
        ops, o = [], 0
        for g in range(world):
            lo, hi = pc[g]
            if g != dst and hi > lo:
                ops += [dist.P2POp(dist.irecv, stage_t[o:o + hi - lo], g),
                        dist.P2POp(dist.irecv, stage_r[o:o + hi - lo], g)]
            o += hi - lo
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        n0, n1, j, k = ch
        o = 0
        for g in range(world):
            lo, hi = pc[g]
            if g == dst or hi == lo:
                continue
            if k == 1:
                off = torch.from_numpy(offs[g, n0:n1 + 1] - offs[g, n0]).to(dev)
                place_node_slice(off, stage_t[o:o + hi - lo], stage_r[o:o + hi - lo], int(bases[g]),
                                 starts[g][n0:n1], out_time, out_rule, engine)
            else:
                d = int(starts_h[g][n0]) + (lo - int(offs[g, n0]))
                out_time[d:d + hi - lo] = stage_t[o:o + hi - lo]
                out_rule[d:d + hi - lo] = stage_r[o:o + hi - lo] + int(bases[g])
            o += hi - lo
    if order == "time" and world > 1:
        rb = np.empty((N, world + 1), dtype=np.int64)
        for g in range(world):
            rb[:, g] = starts_h[g]
        rb[:, world] = node_base.cpu().numpy()[1:]
        merge_rank_runs(rb, out_time, out_rule, engine, budget_bytes)
    return node_base, out_time, out_rule
