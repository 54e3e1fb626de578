"""CPU, world_size 2 over gloo: the sharding and result gather the multi-GPU
bench uses (sedshard.py) — contiguous blocks, no data-path collective, one
gather of fixed-size per-pair results to rank 0."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import sedshard


@pytest.mark.parametrize("total,world", [(10, 2), (7, 3), (64, 8), (3, 4), (0, 2)])
def test_shard_range_partitions(total, world):
    spans = [sedshard.shard_range(total, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = sedshard.shard_range(total, world, rank)
    ids = torch.arange(lo, hi, dtype=torch.int64)
    dist_t = ids.to(torch.float64) * 0.5          # stand-ins for per-pair distance / script length
    len_t = (ids * 3).to(torch.int32)
    got = sedshard.gather_to_rank0([dist_t, len_t], world, rank)
    if rank == 0:
        q.put((got[0].tolist(), got[1].tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 11), (2, 2)])
def test_gather_to_rank0_gloo(world, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    d, ln = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert d == [i * 0.5 for i in range(total)]
    assert ln == [i * 3 for i in range(total)]


def _oracle_distances(strs1, strs2, user):
    """The C oracle as the per-rank distance function (test infrastructure)."""
    import json
    import oracle
    import sedcost
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "user_costs.json" if user else "costs.json")) as f:
        table = json.load(f)
    plan = sedcost.build_plan(table, strs1, strs2)
    cs = oracle.Costs.from_plan(plan)
    return [oracle.pair(cs, plan.encode(a), plan.encode(b), want_ops=False)["dist"] for a, b in zip(strs1, strs2)]


def _avv_worker(rank, world, port, seqs, user, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = sedshard.all_vs_all(seqs, user, world=world, rank=rank, distance_fn=_oracle_distances)
    if rank == 0:
        q.put(got.tolist())
    else:
        assert got is None
    dist.destroy_process_group()


@pytest.mark.parametrize("world,nseq", [(2, 9), (3, 7)])
def test_all_vs_all_row_shards_reassemble(world, nseq):
    """sedshard.all_vs_all over gloo: each rank computes its contiguous block of query rows (here with the
    oracle as the distance function) and rank 0 reassembles the full asymmetric matrix in row order."""
    import numpy as np
    rng = np.random.default_rng(77 + world)
    seqs = ["".join(rng.choice(list("ACGUN"), size=int(rng.integers(1, 30)))) for _ in range(nseq)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_avv_worker, args=(r, world, port, seqs, True, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [_oracle_distances([a] * nseq, seqs, True) for a in seqs]
    assert got == want
