import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "rna-sequence-diff-patch_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def padding_errors(ops, ops_off, len_a, len_b, ln, pairs=None):
    """Pairs whose packed script region (ceil((n+m)/16) words at ops_off[p]) holds a nonzero bit past op ln[p]-1:
    sed.h promises zeros there, in the last op word and in every spare word, on every route."""
    bad = []
    for p in (range(len(ln)) if pairs is None else pairs):
        L = max(int(ln[p]), 0)
        w0, w1 = int(ops_off[p]), int(ops_off[p]) + (int(len_a[p]) + int(len_b[p]) + 15) // 16
        region = ops[w0:w1]
        if L % 16 and int(region[L // 16]) >> (2 * (L % 16)):
            bad.append(p)
        elif region[(L + 15) // 16:].any():
            bad.append(p)
    return bad


@pytest.fixture(scope="session")
def tables():
    return {False: load_golden("costs.json"), True: load_golden("user_costs.json")}


@pytest.fixture(scope="session")
def gpu():
    import sedgpu
    ctx = sedgpu.Context(int(os.environ.get("SED_DEVICE", "0")))
    yield ctx
    ctx.close()
