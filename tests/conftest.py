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


@pytest.fixture(scope="session")
def tables():
    return {False: load_golden("costs.json"), True: load_golden("user_costs.json")}


@pytest.fixture(scope="session")
def gpu():
    import sedgpu
    ctx = sedgpu.Context(int(os.environ.get("SED_DEVICE", "0")))
    yield ctx
    ctx.close()
