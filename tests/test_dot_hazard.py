"""CPU: the v_dot4 result hazard is checked statically in the built library (tools/dot_hazard.py).

The dot-key kernels issue v_dot4_i32_i8 as inline asm, so the compiler inserts no wait states before a reader of
its result; the next instruction reads a stale value (tools/ubench/dot_dist.hip).  These tests fail if a compiler
or flag change ever schedules a v_max3 / v_min3 (or any reader) within 3 wait states of a dot in libsed.so."""
import os
import sys

import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))
import dot_hazard  # noqa: E402

LIB = os.path.join(REPO, "rna-sequence-diff-patch_amd", "libsed.so")

SYNTH = """
0000000000001000 <k>:
\tv_dot4_i32_i8 v81, v49, v18, v53                           // 000000001000: D3A84051 1CD62531
\tv_dot4_i32_i8 v82, v50, v18, v59                           // 000000001008: D3A84052 1CEE2532
\ts_nop 0                                                    // 000000001010: BF800000
\tv_max3_u32 v60, v81, v61, v62                              // 000000001014: D1FA003C 04F67B51
\tv_max3_u32 v63, v82, v60, v64                              // 00000000101C: D1FA003F 05027952
\tv_dot4_i32_i8 v[84:84], v49, v18, v53                      // 000000001024: D3A84051 1CD62531
\tv_mov_b32 v84, 0                                           // 00000000102C: 7EA80280
\tv_dot4_i32_i8 v85, v49, v18, v53                           // 000000001030: D3A84051 1CD62531
\ts_nop 2                                                    // 000000001038: BF800002
\tv_max3_u32 v60, v85, v61, v62                              // 00000000103C: D1FA003C 04F67B51
\tv_dot4_i32_i8 v86, v49, v18, v53                           // 000000001044: D3A84051 1CD62531
\ts_cbranch_scc1 3                                           // 00000000104C: BF850003
\ts_endpgm                                                   // 000000001050: BF810000
"""


def test_scanner_flags_early_readers():
    ndots, closest, viol = dot_hazard.scan([SYNTH])
    assert ndots == 5
    got = [(v[2], v[3]) for v in viol]
    # v81 read after 2 wait states (dot v82 + s_nop 0 = 1 + 1), v82 after 2 (s_nop 0 + max), v86 hits a branch;
    # v84 is overwritten unread, v85 is read after s_nop 2 = 3 wait states
    assert got == [("v81", 2), ("v82", 2), ("v86", 0)], viol
    assert closest == 2


@pytest.mark.skipif(not os.path.exists(LIB), reason="libsed.so not built")
def test_libsed_dot_readers_keep_their_distance():
    ndots, closest, viol = dot_hazard.check(LIB)
    assert ndots > 100  # the dot-key and ladder-dot-key kernels were compiled in
    assert not viol, viol[:10]
