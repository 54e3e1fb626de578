"""CPU: bench.py's multi-GPU plumbing without a GPU — the self-launch command for `--gpus N`, the refusal of a
world size that differs from --gpus or of engine debug switches, and rank 0's verification of every rank's
gathered results (here fed with the oracle's results, then with one corrupted op)."""
import os
import subprocess
import sys
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_launcher_command():
    cmd = bench.launcher_cmd(8, ["--gpus", "8", "--steps", "5"], 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert "--nnodes=1" in cmd
    assert cmd[-4:] == [os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "5"][-4:]
    assert os.path.abspath(cmd[-5]) == os.path.join(REPO, "bench.py")


def test_refuse_reason():
    assert bench.refuse_reason(1, {}) is None
    assert bench.refuse_reason(2, {"WORLD_SIZE": "2"}) is None
    assert "WORLD_SIZE=1" in bench.refuse_reason(2, {"WORLD_SIZE": "1"})
    assert "WORLD_SIZE=4" in bench.refuse_reason(8, {"WORLD_SIZE": "4"})
    assert "SED_DEBUG_NOTB" in bench.refuse_reason(1, {"SED_DEBUG_NOTB": "1"})
    assert bench.refuse_reason(1, {"SED_TBPAR": "0"}) is None  # A/B switches are stamped, not refused


@pytest.mark.parametrize("env,args", [({"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, ["--gpus", "1"]),
                                      ({"WORLD_SIZE": "1"}, ["--gpus", "2"]),
                                      ({"SED_DEBUG_NOTB": "1"}, [])])
def test_bench_refuses_before_touching_the_gpu(env, args):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=e, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 2, r.stderr
    assert "bench.py:" in r.stderr and "{" not in r.stdout


def _pack_ops(ops_list, words):
    out = np.zeros(len(ops_list) * words, np.uint32)
    for p, ops in enumerate(ops_list):
        for k, o in enumerate(ops):
            out[p * words + k // 16] |= np.uint32(int(o) << (2 * (k % 16)))
    return out


def test_verify_gathered_checks_every_rank():
    import json
    import oracle
    import sedcost
    import sedgpu
    from conftest import GOLDEN
    P, n, m, world = 3, 96, 80, 2
    table = json.load(open(os.path.join(GOLDEN, "costs.json")))
    plan = sedcost.build_plan(table, ["ACGU"], ["ACGU"])
    cs = oracle.Costs.from_plan(plan)
    args = SimpleNamespace(workload="c3")
    words = (n + m + 15) // 16
    dists, lens, opsl = [], [], []
    for r in range(world):
        A, B, _, _ = bench.shard_inputs("c3", P, n, m, world, r)
        for p in range(P):
            o = oracle.pair(cs, A[p], B[p])
            dists.append(o["dist"])
            lens.append(o["len"])
            opsl.append(o["ops"])
    gd, gl = np.array(dists), np.array(lens, np.int32)
    go = _pack_ops(opsl, words)
    out = bench.verify_gathered(args, plan, P, n, m, world, gd, gl, go, True, "i32", 2, 5.0)
    assert out["script_valid_rate"] == 1.0 and out["script_exact_rate"] == 1.0
    assert out["verified_on_rank0"]["pairs"] == P * world
    assert out["verified_on_rank0"]["oracle_sample_per_rank"] == [{"pairs": P, "stride": 1}] * 2
    # one op of rank 1's last pair flipped: insert <-> delete keeps the length but breaks the alignment
    bad = [x.copy() for x in opsl]
    k = int(np.argmax(bad[-1] == 2))
    bad[-1][k] = 0
    out = bench.verify_gathered(args, plan, P, n, m, world, gd, gl, _pack_ops(bad, words), True, "i32", 2, 5.0)
    assert out["script_valid_rate"] == pytest.approx(5 / 6) and out["script_exact_rate"] == pytest.approx(5 / 6)
    # a wrong distance on rank 1
    gd2 = gd.copy()
    gd2[P] += 1
    out = bench.verify_gathered(args, plan, P, n, m, world, gd2, gl, go, True, "i32", 2, 5.0)
    assert out["script_valid_rate"] == pytest.approx(5 / 6)


def test_s8d_bytes_config4():
    # SURVEY 8(d) at the config-4 shard: 34.46 GB per launch
    b = bench.s8d_bytes(np.full(8192, 4096), np.full(8192, 4096), True)
    assert abs(b - 34.46e9) < 0.01e9
    assert bench.s8d_bytes([4096], [4096], False) == 2048 + 8


def test_interval_union():
    """The roofline's time basis: overlapping launches (parts on streams, pipelined runs) are counted once."""
    assert bench.interval_union([]) == 0.0
    assert bench.interval_union([(0, 2), (1, 3), (5, 6)]) == pytest.approx(4.0)
    assert bench.interval_union([(5, 6), (0, 10)]) == pytest.approx(10.0)
    assert bench.interval_union([(0, 1), (1, 2), (3, 3)]) == pytest.approx(2.0)  # touching; empty ignored
    # two parts staggered over 3 steps: part 0 [0,7], [10,17], [20,27]; part 1 [3,10], [13,20], [23,30]
    spans = [(10 * k, 10 * k + 7) for k in range(3)] + [(10 * k + 3, 10 * k + 10) for k in range(3)]
    assert bench.interval_union(spans) == pytest.approx(30.0)


def test_strided_sample_spans_the_shard():
    """The exact-rate sample runs first to last pair (every part and residency round), not a prefix."""
    idx, stride = bench.strided_sample(8192, 1100)
    assert stride == 8 and idx[0] == 0 and idx[-1] == 8191
    assert np.all(np.diff(idx) <= stride) and len(idx) == 1025
    assert (idx >= 4096).sum() > 500  # part 1 of the two CK parts
    idx, stride = bench.strided_sample(5, 100)
    assert stride == 1 and list(idx) == [0, 1, 2, 3, 4]
    idx, _ = bench.strided_sample(10, 3)  # stride 4: 0, 4, 8 + the last
    assert list(idx) == [0, 4, 8, 9]


def test_oracle_subset_matches_full_batch():
    import json
    import oracle
    import sedcost
    import sedgpu
    from conftest import GOLDEN
    table = json.load(open(os.path.join(GOLDEN, "user_costs.json")))
    plan = sedcost.build_plan(table, ["ACGU"], ["ACGU"])
    cs = oracle.Costs.from_plan(plan)
    rng = np.random.default_rng(5)
    qa = [rng.integers(0, 4, int(rng.integers(1, 60))).astype(np.uint8) for _ in range(40)]
    qb = [rng.integers(0, 4, int(rng.integers(1, 60))).astype(np.uint8) for _ in range(40)]
    packed = sedgpu.PackedPairs(qa, qb)
    fd, _, fl, fo, foff = oracle.batch(cs, packed.codes_a, packed.off_a, packed.len_a, packed.codes_b, packed.off_b,
                                       packed.len_b, 40, want_ops=True)
    idx, _ = bench.strided_sample(40, 9)
    sd, _, sl, so, soff = bench.oracle_subset(cs, packed, idx, True, 2)
    for k, p in enumerate(idx):
        assert sd[k] == fd[p] and sl[k] == fl[p]
        assert np.array_equal(so[soff[k]:soff[k] + sl[k]], fo[foff[p]:foff[p] + fl[p]])
