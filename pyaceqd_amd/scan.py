"""Sharding of independent propagation units over ranks (one process per GPU).

The reference's only parallelism is a host thread pool of independent ACE processes (one per t1
point or parameter point: correlations.py:153-169, rabi_rotations.py:172-198,
pol_entanglement/G2.py:486-497) — embarrassingly parallel, results gathered in Python lists.
Here the units (t1 points of a two-time sweep, or points of a pulse/B-field scan) are split into
contiguous blocks, one per rank; each rank runs its block as one batched launch on its own GPU and
there is no per-step communication. The only exchange is an optional gather of the finished blocks
to rank 0 (torch.distributed: RCCL over xGMI on the GPU box, gloo on CPU).
"""
import numpy as np


def shard_range(n_units, rank, world):
    """contiguous block [lo, hi) of rank `rank` (sizes differ by at most one)"""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(int(n_units), int(world))
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def shard(units, rank, world):
    lo, hi = shard_range(len(units), rank, world)
    return units[lo:hi]


def gather_blocks(local, dist=None, dst=0):
    """Gather each rank's list of per-unit results (numpy arrays) to `dst` in rank order.
    Returns the concatenated list on dst, None elsewhere (or `local` when not distributed)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return list(local)
    world = dist.get_world_size()
    objs = [None] * world if dist.get_rank() == dst else None
    dist.gather_object([np.asarray(x) for x in local], objs, dst=dst)
    if dist.get_rank() != dst:
        return None
    out = []
    for blk in objs:
        out.extend(blk)
    return out


def gather_tensor(local, dist=None, dst=0):
    """Every rank's 1-D tensor (any length, any device) concatenated in rank order on rank `dst` (None elsewhere).

    One all_gather of the block lengths (8 B per rank), then point-to-point: every other rank sends its block to
    `dst`, which receives each one straight into its slice of the result, on the tensors' own device (RCCL over xGMI
    for GPU tensors, so the result blocks never pass through host memory; gloo for CPU tensors). No padding and no
    copy of any block to the other ranks: at 8 ranks of 655 MB only rank 0 receives, 7 x 655 MB, where an all_gather
    would move 8 x 8 x 655 MB. Complex blocks travel as their real view. This is the one collective of a sharded
    sweep; the reference assembles its result lists from per-process CSV files
    (correlations.py:171-183).

    Round 3 changed this from an all-gather (the result on every rank) to a gather to `dst`: ranks other than `dst`
    now get None. `all_gather_tensor` keeps the old result-on-every-rank behaviour."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return local
    world, rank = dist.get_world_size(), dist.get_rank()
    if not 0 <= dst < world:
        raise ValueError(f"gather_tensor: dst {dst} outside [0, {world})")
    cplx = local.is_complex()
    x = (torch.view_as_real(local) if cplx else local).reshape(-1).contiguous()
    n = torch.tensor([x.numel()], dtype=torch.int64, device=x.device)
    ns = torch.empty(world, dtype=torch.int64, device=x.device)
    dist.all_gather_into_tensor(ns, n)
    sizes = [int(v) for v in ns.tolist()]
    if rank != dst:
        if x.numel():
            dist.send(x, dst)
        return None
    out = torch.empty(sum(sizes), dtype=x.dtype, device=x.device)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    reqs = []
    for r in range(world):
        seg = out[int(offs[r]): int(offs[r + 1])]
        if r == dst:
            seg.copy_(x)
        elif sizes[r]:
            reqs.append(dist.irecv(seg, src=r))
    for q in reqs:
        q.wait()
    return torch.view_as_complex(out.reshape(-1, 2)) if cplx else out


def all_gather_tensor(local, dist=None):
    """Every rank's 1-D tensor concatenated in rank order on EVERY rank (gather_tensor to rank 0, then one broadcast
    of the result): the pre-round-3 semantics of gather_tensor, for callers that use the result on all ranks."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return local
    out = gather_tensor(local, dist, 0)
    cplx = local.is_complex()
    n = torch.tensor([0 if out is None else out.numel()], dtype=torch.int64, device=local.device)
    dist.broadcast(n, 0)
    if out is None:
        out = torch.empty(int(n.item()), dtype=local.dtype, device=local.device)
    buf = torch.view_as_real(out) if cplx else out
    dist.broadcast(buf, 0)
    return out


def triangular_rows(n_t, rank, world):
    """rows [lo, hi) of an upper-triangular pair grid (row i holds the n_t - i pairs (i, i + j), timebin_tl.f90:255-302)
    for `rank`, split so that every rank gets about the same number of pairs (the (i, j) cost is
    about constant per pair, so row i costs n_t - i): boundary b_r is the first row whose cumulative pair count reaches
    r / world of the total"""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    n_t = int(n_t)
    cum = np.concatenate([[0], np.cumsum(np.arange(n_t, 0, -1, dtype=np.int64))])  # pairs in rows [0, i)
    total = int(cum[-1])

    def bound(r):
        if r <= 0:
            return 0
        if r >= world:
            return n_t
        return int(np.searchsorted(cum, r * total / world, side="left"))
    return bound(rank), bound(rank + 1)


def run_sharded(units, work, dist=None):
    """Run `work(block_of_units) -> list of results` on this rank's block and gather to rank 0."""
    if dist is not None and dist.is_initialized():
        rank, world = dist.get_rank(), dist.get_world_size()
    else:
        rank, world = 0, 1
    mine = shard(list(units), rank, world)
    res = work(mine) if len(mine) else []
    return gather_blocks(res, dist)
