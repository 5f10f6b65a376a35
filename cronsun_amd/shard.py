"""Multi-GPU sharding of the expansion.

Rules are independent, so ranks take contiguous job-ID ranges and expand them
with no data-path collective.  The only exchanges are small:

  global_offsets   all-gather of per-rank event totals -> each rank's base
                   offset in the global rule-major CSR
  node_offsets     all-gather of per-node event counts (N int64 per rank) ->
                   offset[g][n] = node_base[n] + sum_{g' < g} count[g'][n], so
                   each node's global list keeps job-ID order across ranks

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
    cuts = [0] + [int(np.searchsorted(c, total * k / world, side="left")) for k in range(1, world)] + [n_rules]
    cuts = np.maximum.accumulate(np.clip(cuts, 0, n_rules))
    return int(cuts[rank]), int(cuts[rank + 1])


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
