"""CPU: the C-ABI library loads, exports exactly what include/sed.h declares,
the ctypes binding covers it, and every entry point fails loudly (no CPU
fallback) when there is no HIP device."""
import ctypes
import os
import re

import pytest

from conftest import REPO
import sedgpu

HEADER = os.path.join(REPO, "include", "sed.h")


def declared():
    src = open(HEADER).read()
    return re.findall(r"^[a-z_0-9 ]+?\**\s*\**(sed_[a-z_0-9]+)\(", src, re.M)


def test_library_exports_every_declared_symbol():
    names = declared()
    assert len(names) >= 20
    lib = ctypes.CDLL(sedgpu.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    bound = {name for name, _, _ in sedgpu.SIGNATURES}
    assert set(declared()) == bound


def test_version_string():
    assert sedgpu.load().sed_version().startswith(b"libsed")


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(sedgpu.SedError):
        sedgpu.Context(0)


def test_null_context_is_rejected():
    lib = sedgpu.load()
    assert lib.sed_set_option(None, 1, 0) == -1
    assert lib.sed_last_error(None) == b"null context"
