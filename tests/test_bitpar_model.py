"""CPU: the bit-parallel recurrence of the unit-cost lane kernels (sed_lane.hip: sed_lane_bitpar_kernel and the
flagged pairs of sed_lane_f64_kernel), restated word op by word op in Python, against the C oracle's distances
under costs.json's unit ACGU costs (insert = delete = 1, every mismatch 1).  It pins the kernel's formulation
(bit planes of the 2-bit codes, the top border's +1 as the carry-in of the shifted Ph, the sink as
n + popcount(Pv) - popcount(Mv) over bits 0..m-1, don't-care bits at and above m) before any GPU runs it."""
import numpy as np
import pytest

import oracle
import sedcost
from conftest import load_golden

M32 = 0xFFFFFFFF


def bitpar_distance(a, b):
    """a: str1 codes (rows, any length), b: str2 codes (bit dimension, 1..32), codes 0..3."""
    m, n = len(b), len(a)
    E0 = E1 = 0
    for j, c in enumerate(b):
        E0 |= (c & 1) << j
        E1 |= (c >> 1) << j
    Pv, Mv = M32, 0
    for c in a:
        c0 = M32 if c & 1 else 0  # (the kernel: v_bfe_i32 of the packed word)
        c1 = M32 if c & 2 else 0
        tq = (E0 ^ c0) | (E1 ^ c1)  # ~Eq
        Xv = (Mv | ~tq) & M32
        Xh = ((((Pv & ~tq) + Pv) & M32) ^ Pv) | (~tq & M32)
        Ph = (((Mv | ~(Xh | Pv)) << 1) | 1) & M32
        Mh = ((Pv & Xh) << 1) & M32
        Pv = (Mh | ~(Xv | Ph)) & M32
        Mv = Ph & Xv
    keep = M32 if m >= 32 else (1 << m) - 1
    return n + bin(Pv & keep).count("1") - bin(Mv & keep).count("1")


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_bitpar_recurrence_vs_oracle(seed):
    table = load_golden("costs.json")  # its ACGU block is unit cost
    rng = np.random.default_rng(900 + seed)
    pairs = []
    for _ in range(400):
        n = int(rng.choice([rng.integers(1, 40), rng.integers(1, 513)]))
        m = int(rng.choice([rng.integers(1, 33), 32, 1, 16, 17]))
        a = "".join(rng.choice(list("ACGU"), size=n))
        b = "".join(c if rng.random() > 0.1 else rng.choice(list("ACGU")) for c in (a * 40)[:m]) \
            if rng.random() < 0.4 else "".join(rng.choice(list("ACGU"), size=m))
        pairs.append((a, b))
    pairs += [("A", "A"), ("A", "C"), ("G" * 512, "G" * 32), ("ACGU" * 128, "U"), ("U", "ACGU" * 8)]
    plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
    cs = oracle.Costs.from_plan(plan)
    for a, b in pairs:
        ea, eb = plan.encode(a), plan.encode(b)
        want = oracle.pair(cs, ea, eb, want_ops=False)["dist"]
        # any 2-bit code assignment works: the plan's codes of A, C, G, U
        assert float(bitpar_distance([int(x) for x in ea], [int(x) for x in eb])) == want, (a, b)
