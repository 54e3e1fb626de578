"""CPU: the signed-byte factorisations behind the dot keys (sed_runtime.cpp: dot_keys, via sed_dot_factor).
The checkpoint forward kernel adds dot4(row(a), col(b)) = A*kappa(a, b) + 1 to the diagonal and maximises; the
CHAIN kernel's ladder keys add -(A*kappa + u - 1) (u = 16 on the wide ladder, else 8).  Checked here for both shipped tables: exact products, byte ranges,
the ordering bound A > min(n, m) (kmax - kmin) / kmin, the decode multiply-shift, and the ineligible cases."""
import numpy as np
import pytest

from conftest import load_golden
import sedgpu

S = "ACGU"


def _table(name):
    t = load_golden(name)
    sub = np.array([[0.0 if a == b else t["update"][a][b] for b in S] for a in S])
    return sub, t["insert"], t["delete"]


@pytest.mark.parametrize("name, maxmin, want_A", [("user_costs.json", 4096, 2880), ("costs.json", 4096, 12700)])
def test_dot_keys_factorisation(name, maxmin, want_A):
    sub, ins, dele = _table(name)
    got = sedgpu.dot_factor(sub, ins, dele, maxmin=maxmin)
    assert got is not None
    A, rows, cols, (shift, mult) = got
    assert A == want_A
    kap = (ins + dele - sub).astype(np.int64)
    assert np.array_equal(rows @ cols.T, A * kap + 1)  # v_dot4_i32_i8 of row and column vectors
    assert np.abs(rows).max() <= 127 and np.abs(cols).max() <= 127
    kmin, kmax = kap.min(), kap.max()
    assert A * kmin > maxmin * (kmax - kmin)  # candidates' U spread below A
    # decode X = floor(k kmax / (A kmax + 1)) by (k * mult) >> shift on keys k = A X + U of real paths
    rng = np.random.default_rng(1)
    for _ in range(20000):
        U = int(rng.integers(0, maxmin + 1))
        X = int(rng.integers(U * kmin, U * kmax + 1))
        k = A * X + U
        assert (k * mult) >> shift == X and k - A * X == U


def test_dot_keys_bound_and_ladder_eligibility():
    sub, ins, dele = _table("user_costs.json")
    assert sedgpu.dot_factor(sub, ins, dele, maxmin=4319) is not None
    assert sedgpu.dot_factor(sub, ins, dele, maxmin=4320) is None  # 2880 * 3 <= 4320 * 2
    assert sedgpu.dot_factor(sub, ins, dele, ladder_maxsum=1024) is None  # A > 8 (n + m) does not fit bytes
    sub, ins, dele = _table("costs.json")
    kap = (ins + dele - sub).astype(np.int64)
    # config 3 (512 x 512): the wide ladder, A > 16 min(n, m) + 15 (its sink decode reads L inside [max, n + m])
    A, rows, cols, (sent, unit) = sedgpu.dot_factor(sub, ins, dele, maxmin=512, ladder_maxsum=1024)
    assert unit == 16 and A % 16 == 0 and 16 * 512 + 15 < A < 65536
    assert np.array_equal(rows @ cols.T, -(A * kap + 15))  # min-form ladder keys: negated column vectors
    assert 16 <= sent * rows[0, 0] <= 480 and np.all(rows[:, 0] == rows[0, 0])  # the sentinel column {s, 0, 0, 0}
    # where the wide ladder's A does not fit bytes (A > 16 * 1024 + 15 here), the 3-bit ladder's: A > 8 (n + m) + 7
    A8, rows8, cols8, (sent8, unit8) = sedgpu.dot_factor(sub, ins, dele, ladder_maxsum=1024)
    assert unit8 == 8 and A8 % 8 == 0 and 8 * 1024 + 7 < A8 < 65536
    assert np.array_equal(rows8 @ cols8.T, -(A8 * kap + 7)) and 8 <= sent8 * rows8[0, 0] <= 490
    fractional = sub.copy()
    fractional[0, 1] = 0.5
    assert sedgpu.dot_factor(fractional, ins, dele, maxmin=100) is None


def test_ladder_unit_is_a_multiple_of_8_on_random_tables():
    """Ladder dot keys keep the rung and the op in the low 3 (wide: 4) bits of A*(D - i*delete - j*insert) + u*(L - i
    - j) + B + c(i), u = 8 (16): every ladder factorisation must have A % u == 0 (a random insert 2 / delete 1 table
    once factored with A = 8835 and produced wrong scripts on the GPU), A within 16 bits and above u (n + m) + u - 1,
    and exact bytes."""
    rng = np.random.default_rng(91)
    seen = 0
    for _ in range(3000):
        ins, de = int(rng.integers(1, 4)), int(rng.integers(1, 4))
        sub = rng.integers(1, min(2, ins + de) + 1, size=(4, 4)).astype(float)
        np.fill_diagonal(sub, 0)
        got = sedgpu.dot_factor(sub, ins, de, 0, 1024)
        if got is None:
            continue
        seen += 1
        A, rows, cols, (_, u) = got
        assert u in (8, 16) and A % u == 0 and u * 1024 + u - 1 < A < 65536
        kap = ins + de - sub
        assert np.array_equal(rows @ cols.T, -(A * kap + u - 1))
    assert seen >= 3
