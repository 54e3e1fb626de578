"""TEST INFRASTRUCTURE — ctypes binding of oracle/liboracle.so (sed_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module; the product path (libsed.so through sedgpu.py) never does.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class _Costs(C.Structure):
    _fields_ = [("K", C.c_int), ("sub", C.POINTER(C.c_double)), ("sub_int", C.POINTER(C.c_uint8)),
                ("ins", C.c_double), ("dele", C.c_double), ("ins_int", C.c_int), ("del_int", C.c_int)]


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", HERE])
        lib = C.CDLL(LIB_PATH)
        P = C.c_void_p
        lib.sed_oracle_pair.argtypes = [P, C.c_int, P, C.c_int, C.POINTER(_Costs), C.POINTER(C.c_double),
                                        C.POINTER(C.c_int), C.POINTER(C.c_int), P, P, P, P]
        lib.sed_oracle_pair.restype = C.c_int
        lib.sed_oracle_batch.argtypes = [P, P, P, P, P, P, C.c_int, C.POINTER(_Costs), P, P, P, P, P, C.c_int]
        lib.sed_oracle_batch.restype = C.c_int
        lib.sed_synth_codes.argtypes = [C.c_uint64, C.c_uint64, C.c_int, C.c_int, P]
        lib.sed_synth_codes.restype = None
        _lib = lib
    return _lib


class Costs:
    """Resolved K x K cost model (same meaning as sedcost.CostPlan)."""

    def __init__(self, sub, sub_int, ins, ins_int, dele, del_int):
        self.sub = np.ascontiguousarray(sub, np.float64)
        self.sub_int = np.ascontiguousarray(sub_int, np.uint8)
        self.c = _Costs(self.sub.shape[0], self.sub.ctypes.data_as(C.POINTER(C.c_double)),
                        self.sub_int.ctypes.data_as(C.POINTER(C.c_uint8)), ins, dele, ins_int, del_int)

    @classmethod
    def from_plan(cls, plan):
        return cls(plan.sub, plan.sub_int, plan.ins, plan.ins_int, plan.dele, plan.del_int)


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def pair(costs, a, b, want_ops=True, full=False):
    """dist, is_int, len, ops (uint8 codes) [, D, T, M full matrices]."""
    lib = load()
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    n, m = len(a), len(b)
    dist, ii, ln = C.c_double(), C.c_int(), C.c_int()
    ops = np.zeros(max(n + m, 1), np.uint8) if want_ops else None
    D = T = M = None
    if full:
        D = np.zeros((n + 1, m + 1), np.float64)
        T = np.zeros((n + 1, m + 1), np.uint8)
        M = np.zeros((n + 1, m + 1), np.uint8)
    rc = lib.sed_oracle_pair(_ptr(a) if n else None, n, _ptr(b) if m else None, m, C.byref(costs.c), C.byref(dist),
                             C.byref(ii), C.byref(ln), _ptr(ops) if want_ops else None,
                             _ptr(D) if full else None, _ptr(T) if full else None, _ptr(M) if full else None)
    if rc:
        raise MemoryError("oracle allocation failed")
    out = {"dist": dist.value, "is_int": ii.value, "len": ln.value}
    if want_ops:
        out["ops"] = ops[:ln.value].copy()
    if full:
        out.update(D=D, T=T, M=M)
    return out


def batch(costs, codes_a, off_a, len_a, codes_b, off_b, len_b, npairs, want_ops=False, nthreads=1):
    lib = load()
    dist = np.zeros(max(npairs, 1), np.float64)
    is_int = np.zeros(max(npairs, 1), np.int32)
    ln = np.zeros(max(npairs, 1), np.int32)
    ops = ops_off = None
    if want_ops:
        ops_off = np.zeros(max(npairs, 1), np.int64)
        tot = (np.asarray(len_a[:npairs], np.int64) + np.asarray(len_b[:npairs], np.int64))
        if npairs:
            ops_off[1:npairs] = np.cumsum(tot[:-1])
        ops = np.zeros(max(int(tot.sum()), 1), np.uint8)
    rc = lib.sed_oracle_batch(_ptr(codes_a), _ptr(off_a), _ptr(len_a), _ptr(codes_b), _ptr(off_b), _ptr(len_b),
                              npairs, C.byref(costs.c), _ptr(dist), _ptr(is_int), _ptr(ln),
                              _ptr(ops) if want_ops else None, _ptr(ops_off) if want_ops else None, nthreads)
    if rc:
        raise MemoryError("oracle allocation failed")
    return dist[:npairs], is_int[:npairs], ln[:npairs], ops, ops_off


def synth_codes(base, pair_id, stream, length):
    out = np.zeros(max(length, 1), np.uint8)
    load().sed_synth_codes(base, pair_id, stream, length, _ptr(out))
    return out[:length]


OPCH = "idu"


def ops_to_str(ops):
    return "".join(OPCH[int(o)] for o in ops)
