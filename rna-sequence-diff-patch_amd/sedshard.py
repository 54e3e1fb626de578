"""Multi-GPU sharding for batches of independent pairs.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
MI355X).  Pairs are independent, so the data path has no collective: rank r
takes a contiguous block of pair (or query-row) indices, generates or loads its
own inputs, runs the engine, and only the fixed-size per-pair results travel,
once, to rank 0 (gather_to_rank0).  The same code runs over gloo on CPU tensors
for the tests.
"""
import numpy as np


def shard_range(total, world, rank):
    """[start, stop) of a contiguous, near-equal block of `total` items for `rank`."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_to_rank0(tensors, world, rank):
    """Gather 1-D tensors of per-rank length to rank 0 (pad to the max length,
    gather, trim).  Returns, on rank 0, one concatenated tensor per input; None elsewhere."""
    import torch
    import torch.distributed as dist
    n_local = torch.tensor([t.numel() for t in tensors], dtype=torch.int64, device=tensors[0].device)
    sizes = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(sizes, n_local)
    sizes = torch.stack(sizes).cpu()
    out = []
    for k, t in enumerate(tensors):
        width = int(sizes[:, k].max())
        buf = torch.zeros(width, dtype=t.dtype, device=t.device)
        buf[:t.numel()] = t
        parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
        dist.gather(buf, parts, dst=0)
        if rank == 0:
            out.append(torch.cat([p[:int(sizes[r, k])] for r, p in enumerate(parts)]))
    return out if rank == 0 else None


def all_vs_all(seqs, userCosts=False, world=1, rank=0, device=None, distance_fn=None):
    """Row block of the len(seqs) x len(seqs) matrix of dp[n][m].value
    (query = row = str1, document = column = str2, as IRMethods.search_collection
    orders them) computed on this rank's GPU, gathered to rank 0 as a float64
    numpy matrix (None on other ranks).  One engine launch per rank.
    distance_fn(strs1, strs2, userCosts) -> values replaces StringEditDistance.distance_batch
    (the CPU tests inject the oracle to check the sharding and reassembly)."""
    import torch
    if distance_fn is None:
        import StringEditDistance as SED
        distance_fn = SED.distance_batch
    lo, hi = shard_range(len(seqs), world, rank)
    q = [a for a in seqs[lo:hi] for _ in seqs]
    d = [b for _ in seqs[lo:hi] for b in seqs]
    vals = np.array(distance_fn(q, d, userCosts), dtype=np.float64) if q else np.zeros(0)
    if world == 1:
        return vals.reshape(hi - lo, len(seqs))
    t = torch.from_numpy(vals).to(device if device is not None else "cpu")
    got = gather_to_rank0([t], world, rank)
    if rank != 0:
        return None
    return got[0].cpu().numpy().reshape(len(seqs), len(seqs))
