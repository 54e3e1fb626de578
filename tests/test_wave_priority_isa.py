"""CPU: the built code object carries the round-5 wave priorities (DESIGN "Wave priorities"): the kernels that share
SIMDs by design set their issue priority with s_setprio, and the config-4 forward does not.

- sed_traceback_ck_kernel (the checkpoint traceback beside the other part's forward): s_setprio 1
  (SED_CKTB_PRIO; c4 9.74-9.86 against 9.91-10.32 ms at 0, profiles/r05/s15, s16);
- sed_traceback_kernel (per-cell codes, integer batches only: a uniform branch on its ladder pattern): s_setprio 1;
- sed_wf_f64_kernel (the fp64 DP beside the previous run's traceback): s_setprio 1;
- the SPLIT forwards (config 2's stripe waves, and the fp64 SPLIT route's): s_setprio 2;
- the checkpoint forward sed_wf_i32_kernel<16, ..., CK, DOT>: none (its waves must yield to the traceback's).
A build with other -DSED_*_PRIO values, or a compiler that drops the builtin, fails here."""
import os
import sys
import tempfile

import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))
import dot_hazard  # noqa: E402

LIB = os.path.join(REPO, "rna-sequence-diff-patch_amd", "libsed.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="libsed.so not built")
def test_wave_priorities_in_code_object():
    with tempfile.TemporaryDirectory(prefix="prioisa_") as wd:
        texts = dot_hazard.disassemble(LIB, wd)
    prio = {}  # kernel symbol -> set of s_setprio operands
    seen = set()
    for t in texts:
        for line in t.split("\n"):
            s = line.strip()
            if s.endswith(">:") and "<" in s:
                cur = s[s.index("<") + 1:-2]
                seen.add(cur)
            elif s.startswith("s_setprio"):
                prio.setdefault(cur, set()).add(s.split()[1])
    def of(prefix):
        ks = [k for k in seen if k.startswith(prefix)]
        assert ks, prefix
        return ks
    for k in of("_Z23sed_traceback_ck_kernelILi16E"):
        assert prio.get(k) == {"1"}, (k, prio.get(k))
    for k in of("_Z20sed_traceback_kernelILi8ELi64E"):
        assert prio.get(k) == {"1"}, (k, prio.get(k))
    for k in of("_Z17sed_wf_f64_kernelILi8ELb1E"):
        assert prio.get(k) == {"1"}, (k, prio.get(k))
    for k in of("_Z17sed_wf_i32_kernelILi4ELb0ELb1ELb0ELb1ELb1E"):  # SPLIT, checkpoints, dot keys (config 2)
        assert prio.get(k) == {"2"}, (k, prio.get(k))
    for k in of("_Z17sed_wf_i32_kernelILi16ELb0ELb0ELb0ELb1ELb1E"):  # the config-4 forward
        assert not prio.get(k), (k, prio.get(k))
    for k in of("_Z23sed_wf_f64_split_kernelILi2E"):  # fp64 SPLIT: its stripe waves are latency-bound too
        assert prio.get(k) == {"2"}, (k, prio.get(k))
