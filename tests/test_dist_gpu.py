"""GPU: the result gather of the multi-GPU bench over RCCL (backend "nccl").

The one-GPU box cannot run two RCCL ranks (RCCL refuses two ranks on one device), so this runs the
rank-0 side of the exchange as world size 1 in a spawned process: process-group init with the device
bound, the all_gather of per-rank sizes and the padded dist.gather of the three result tensors
(float64 distances, int32 lengths, int32 script words) that bench.py sends, plus the MAX/SUM
all-reduces of its timing and cell count.  The N > 1 data movement itself is covered over gloo
(tests/test_dist.py)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import sedshard

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank0(port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        dev = torch.device("cuda", 0)
        d = torch.arange(37, dtype=torch.float64, device=dev) * 0.25
        ln = torch.arange(37, dtype=torch.int32, device=dev) * 3
        ops = torch.arange(1001, dtype=torch.int32, device=dev) - 500
        got = sedshard.gather_to_rank0([d, ln, ops], 1, 0)
        t = torch.tensor([1.5], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        c = torch.tensor([7.0], dtype=torch.float64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        torch.cuda.synchronize()
        q.put(([g.cpu().tolist() for g in got], float(t.item()), float(c.item())))
    finally:
        dist.destroy_process_group()


def test_gather_to_rank0_rccl_world1():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank0, args=(_free_port(), q))
    p.start()
    got, tmax, csum = q.get(timeout=100)
    p.join(timeout=30)
    assert p.exitcode == 0
    assert got[0] == [i * 0.25 for i in range(37)]
    assert got[1] == [i * 3 for i in range(37)]
    assert got[2] == [i - 500 for i in range(1001)]
    assert tmax == 1.5 and csum == 7.0
