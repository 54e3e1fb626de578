"""GPU: the C-ABI's error contract (include/sed.h): negative return codes and a message, never
an exception across the ABI, never a silent fallback; the context stays usable afterwards."""
import numpy as np
import pytest

import sedcost
import sedgpu

pytestmark = pytest.mark.gpu


def _packed(a, b):
    return sedgpu.PackedPairs([np.asarray(a, np.uint8)], [np.asarray(b, np.uint8)])


def test_costs_must_be_set_first():
    ctx = sedgpu.Context(0)
    try:
        with pytest.raises(sedgpu.SedError, match="sed_set_costs"):
            ctx.run(_packed([0, 1], [1, 0]), False)
    finally:
        ctx.close()


def test_errors_leave_the_context_usable(gpu, tables):
    plan = sedcost.build_plan(tables[False], ["ACGU"], ["ACGU"])
    gpu.set_costs(plan)
    # symbol code outside the alphabet
    with pytest.raises(sedgpu.SedError, match="code 9 >= K"):
        gpu.run(_packed([0, 9], [1]), False)
    # forced integer kernel with costs it cannot represent (IUPAC fractions)
    iupac = sedcost.build_plan(tables[False], ["AGCUYRWSKMDVHBN"], ["AGCUYRWSKMDVHBN"])
    gpu.set_costs(iupac)
    gpu.set_mode(1)
    try:
        with pytest.raises(sedgpu.SedError, match="not eligible"):
            gpu.run(_packed([0, 4], [1, 5]), False)
    finally:
        gpu.set_mode(0)
    # forced integer kernel whose packed key would overflow (D >= 2^16 - 256)
    gpu.set_costs(plan)
    gpu.set_mode(1)
    try:
        with pytest.raises(sedgpu.SedError, match="overflow"):
            gpu.run(_packed(np.zeros(70000, np.uint8), np.ones(1, np.uint8)), False)
    finally:
        gpu.set_mode(0)
    # ... and the auto mode takes the fp64 kernel for that pair instead
    d, ii, ln, _ = gpu.run(_packed(np.zeros(70000, np.uint8), np.ones(1, np.uint8)), False)
    assert d[0] == 70000.0 and ln[0] == 70000
    # the context still works
    d, ii, ln, _ = gpu.run(_packed([0, 1, 2], [0, 1, 2]), True)
    assert d[0] == 0.0 and ii[0] == 1 and ln[0] == 3


def test_alphabet_limit_and_bad_options(gpu):
    K = 40
    lib = gpu._lib
    sub = np.ones(K * K, np.float64)
    sub_int = np.zeros(K * K, np.uint8)
    assert lib.sed_set_costs(gpu.ptr, K, sub, sub_int, 1.0, 0, 1.0, 0) == 0
    gpu.invalidate_costs()
    with pytest.raises(sedgpu.SedError, match="exceeds"):
        gpu.run(_packed([1, 39], [2]), False)
    assert lib.sed_set_option(gpu.ptr, sedgpu.SED_OPT_ROWS_PER_LANE, 3) == -1
    assert lib.sed_set_option(gpu.ptr, 99, 0) == -1
    assert b"bad option" in lib.sed_last_error(gpu.ptr)


def test_batch_state_errors(gpu, tables):
    plan = sedcost.build_plan(tables[False], ["ACGU"], ["ACGU"])
    gpu.set_costs(plan)
    b = sedgpu.Batch(gpu, _packed([0, 1], [1, 0]), True)
    try:
        with pytest.raises(sedgpu.SedError, match="not been run"):
            b.results()
        b.run()
        d, ii, ln, ops = b.results()
        assert d[0] == 2.0 and ln[0] == 2
    finally:
        b.close()
