"""CPU: the config-4 forward kernel keeps no register copies of its row state in the chunk loop.

sed_wf_i32_kernel<16, TB=0, SPLIT=0, LEN=0, CK=1, DOT=1> is the headline forward.  When one loop chose
per chunk between the unrolled group body and the rolled (sink) body, the register allocator copied the 16 row
values between the two bodies' registers at every chunk end (16 v_mov_b64 on each side of the merge: 34 in the
kernel, ~24 VALU per 2112 in the hot loop).  The chunks before the sink now run a loop of their own and the kernel
has 2 (profiles/r04/s14: c4 9.80 against 9.92 ms).  This test reads the built code object (the disassembler that
tools/dot_hazard.py uses) and fails if a compiler or source change brings the copies back."""
import os
import sys
import tempfile

import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))
import dot_hazard  # noqa: E402

LIB = os.path.join(REPO, "rna-sequence-diff-patch_amd", "libsed.so")
KERNEL = "_Z17sed_wf_i32_kernelILi16ELb0ELb0ELb0ELb1ELb1E"


@pytest.mark.skipif(not os.path.exists(LIB), reason="libsed.so not built")
def test_ck_forward_has_no_row_state_copies():
    with tempfile.TemporaryDirectory(prefix="ckisa_") as wd:
        texts = dot_hazard.disassemble(LIB, wd)
    ins = [(fn, mn) for t in texts for fn, mn, _ in dot_hazard.parse(t) if fn and fn.startswith(KERNEL)]
    assert ins, "the R = 16 checkpoint forward kernel is not in libsed.so"
    count = {}
    for _, mn in ins:
        count[mn] = count.get(mn, 0) + 1
    assert count.get("v_dot4_i32_i8", 0) >= 128  # two unrolled groups of 4 steps x 16 rows, at least
    movs64 = sum(v for mn, v in count.items() if mn.startswith("v_mov_b64"))  # v_mov_b64_e32 in objdump's spelling
    assert movs64 <= 4, movs64
