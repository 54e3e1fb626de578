"""ctypes binding of libsed.so (include/sed.h) — the only way the Python side
reaches the GPU engine.  There is deliberately no CPU fallback: if the library
or a HIP device is missing, every entry point raises.
"""
import ctypes as C
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SED_LIBRARY", os.path.join(HERE, "libsed.so"))

SED_WANT_SCRIPT = 1
SED_PIPELINE = 2
SED_NO_LEN = 4
SED_OPT_MODE = 1
SED_OPT_ROWS_PER_LANE = 2
SED_OPT_SPLIT = 3
SED_OPT_LANE = 4
SED_OPT_CHAIN = 5
SED_OPT_PACK = 6
SED_OPT_TB = 7
SED_OPT_CHAIN_WAVES = 8
SED_OPT_DEBUG_CORRUPT = 9
MODE_NAMES = {1: "i32", 2: "f64", 3: "f64-typed"}

_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")

# (name, restype, argtypes) — every symbol include/sed.h declares
SIGNATURES = [
    ("sed_version", C.c_char_p, []),
    ("sed_create", C.c_void_p, [C.c_int]),
    ("sed_destroy", None, [C.c_void_p]),
    ("sed_last_error", C.c_char_p, [C.c_void_p]),
    ("sed_set_option", C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    ("sed_set_costs", C.c_int, [C.c_void_p, C.c_int, _f64p, _u8p, C.c_double, C.c_int, C.c_double, C.c_int]),
    ("sed_run_batch", C.c_int, [C.c_void_p, _u8p, _i64p, _i32p, _u8p, _i64p, _i32p, C.c_int32, C.c_uint32,
                                _f64p, _u8p, _i32p, C.c_void_p, C.c_void_p]),
    ("sed_batch_create", C.c_void_p, [C.c_void_p, _u8p, _i64p, _i32p, _u8p, _i64p, _i32p, C.c_int32, C.c_uint32]),
    ("sed_batch_destroy", None, [C.c_void_p]),
    ("sed_batch_mode", C.c_int, [C.c_void_p]),
    ("sed_batch_rows_per_lane", C.c_int, [C.c_void_p]),
    ("sed_batch_lane_pairs", C.c_int, [C.c_void_p]),
    ("sed_batch_chains", C.c_int, [C.c_void_p]),
    ("sed_batch_packed_pairs", C.c_int, [C.c_void_p]),
    ("sed_batch_traceback_mode", C.c_int, [C.c_void_p]),
    ("sed_batch_chain_stats", C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("sed_batch_run", C.c_int, [C.c_void_p]),
    ("sed_batch_sync", C.c_int, [C.c_void_p]),
    ("sed_batch_last_times", C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    ("sed_batch_times", C.c_int, [C.c_void_p, _f32p, _f32p, C.c_int]),
    ("sed_batch_reset_times", C.c_int, [C.c_void_p]),
    ("sed_batch_results", C.c_int, [C.c_void_p, _f64p, _u8p, _i32p, C.c_void_p, C.c_void_p]),
    ("sed_batch_device_results", C.c_int, [C.c_void_p] + [C.POINTER(C.c_uint64)] * 5),
    ("sed_batch_export", C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64]),
    ("sed_batch_work", C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    ("sed_selftest", C.c_int, [C.c_void_p]),
    ("sed_full_matrix", C.c_int, [C.c_void_p, _u8p, C.c_int32, _u8p, C.c_int32, _f64p, _u8p]),
]

_lib = None
_lock = threading.Lock()


class SedError(RuntimeError):
    pass


def load():
    """Load libsed.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SedError("libsed.so not found at %s: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                       % LIB_PATH)
    lib = C.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


class Context:
    """One sed_ctx (device + stream + cost table)."""

    def __init__(self, device=0):
        lib = load()
        self._lib = lib
        self.ptr = lib.sed_create(device)
        if not self.ptr:
            raise SedError("sed_create(%d) failed: no usable HIP device" % device)
        self._cost_key = None

    def close(self):
        if self.ptr:
            self._lib.sed_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = self._lib.sed_last_error(self.ptr)
            raise SedError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))

    def set_option(self, key, value):
        self._check(self._lib.sed_set_option(self.ptr, key, value), "sed_set_option")

    def set_mode(self, mode):
        """0 auto, 1 integer, 2 fp64, 3 fp64 with int typing."""
        self.set_option(SED_OPT_MODE, mode)
        self._cost_key = None

    def set_costs(self, plan):
        key = plan.key()
        if key == self._cost_key:
            return
        sub = np.ascontiguousarray(plan.sub, dtype=np.float64).ravel()
        sub_int = np.ascontiguousarray(plan.sub_int, dtype=np.uint8).ravel()
        self._check(self._lib.sed_set_costs(self.ptr, plan.K, sub, sub_int, plan.ins, plan.ins_int,
                                            plan.dele, plan.del_int), "sed_set_costs")
        self._cost_key = key

    def selftest(self):
        return self._lib.sed_selftest(self.ptr)

    def run(self, packed, want_script, no_len=False):
        """packed: PackedPairs.  Returns (dist f64[], is_int u8[], len i32[], ops u32[] | None).
        no_len (distance only): lengths are not computed (-1), the integer kernels run 3 ops/cell."""
        np_ = packed.npairs
        dist = np.zeros(max(np_, 1), np.float64)
        is_int = np.zeros(max(np_, 1), np.uint8)
        ln = np.zeros(max(np_, 1), np.int32)
        ops = None
        ops_ptr = ops_off_ptr = None
        if want_script:
            ops = np.zeros(max(int(packed.ops_off[-1]), 1), np.uint32)
            ops_ptr = ops.ctypes.data_as(C.c_void_p)
            ops_off_ptr = packed.ops_off.ctypes.data_as(C.c_void_p)
        rc = self._lib.sed_run_batch(self.ptr, packed.codes_a, packed.off_a, packed.len_a, packed.codes_b,
                                     packed.off_b, packed.len_b, np_,
                                     SED_WANT_SCRIPT if want_script else (SED_NO_LEN if no_len else 0),
                                     dist, is_int, ln, ops_ptr, ops_off_ptr)
        self._check(rc, "sed_run_batch")
        return dist[:np_], is_int[:np_], ln[:np_], ops

    def full_matrix(self, codes_a, codes_b):
        n, m = len(codes_a), len(codes_b)
        D = np.zeros((n + 1) * (m + 1), np.float64)
        M = np.zeros((n + 1) * (m + 1), np.uint8)
        rc = self._lib.sed_full_matrix(self.ptr, np.ascontiguousarray(codes_a, np.uint8) if n else np.zeros(1, np.uint8),
                                       n, np.ascontiguousarray(codes_b, np.uint8) if m else np.zeros(1, np.uint8),
                                       m, D, M)
        self._check(rc, "sed_full_matrix")
        return D.reshape(n + 1, m + 1), M.reshape(n + 1, m + 1)


class PackedPairs:
    """Concatenated codes + offsets for a list of (codes_a, codes_b) pairs."""

    def __init__(self, pairs_a, pairs_b):
        self.npairs = len(pairs_a)
        self.len_a = np.array([len(x) for x in pairs_a] or [0], dtype=np.int32)
        self.len_b = np.array([len(x) for x in pairs_b] or [0], dtype=np.int32)
        self.off_a = np.zeros(max(self.npairs, 1), np.int64)
        self.off_b = np.zeros(max(self.npairs, 1), np.int64)
        if self.npairs:
            self.off_a[1:] = np.cumsum(self.len_a[:-1])
            self.off_b[1:] = np.cumsum(self.len_b[:-1])
        self.codes_a = np.concatenate([np.asarray(x, np.uint8) for x in pairs_a] + [np.zeros(1, np.uint8)])
        self.codes_b = np.concatenate([np.asarray(x, np.uint8) for x in pairs_b] + [np.zeros(1, np.uint8)])
        words = (self.len_a.astype(np.int64) + self.len_b + 15) // 16
        self.ops_off = np.zeros(max(self.npairs, 1) + 1, np.int64)
        if self.npairs:
            self.ops_off[1:self.npairs + 1] = np.cumsum(words[:self.npairs])

    @classmethod
    def from_arrays(cls, A, B):
        """Fixed-length pairs from 2-D uint8 arrays (npairs x n), (npairs x m)."""
        self = cls.__new__(cls)
        P, n = A.shape
        m = B.shape[1]
        self.npairs = P
        self.len_a = np.full(max(P, 1), n, np.int32)
        self.len_b = np.full(max(P, 1), m, np.int32)
        self.off_a = (np.arange(max(P, 1), dtype=np.int64) * n)
        self.off_b = (np.arange(max(P, 1), dtype=np.int64) * m)
        self.codes_a = np.ascontiguousarray(np.concatenate([A.ravel(), np.zeros(1, np.uint8)]), np.uint8)
        self.codes_b = np.ascontiguousarray(np.concatenate([B.ravel(), np.zeros(1, np.uint8)]), np.uint8)
        w = (n + m + 15) // 16
        self.ops_off = np.arange(max(P, 1) + 1, dtype=np.int64) * w
        return self


def unpack_ops(ops_words, ops_off, p, length):
    """Op codes (uint8 0 ins, 1 del, 2 upd) of pair p from the packed script buffer."""
    w = ops_words[ops_off[p]: ops_off[p] + (length + 15) // 16]
    codes = (w[:, None] >> (2 * np.arange(16, dtype=np.uint32))[None, :]) & 3
    return codes.ravel()[:length].astype(np.uint8)


class Batch:
    """Device-resident batch (sed_batch_*): upload once, run many times."""

    def __init__(self, ctx, packed, want_script, pipeline=False, no_len=False):
        self.ctx = ctx
        self._lib = ctx._lib
        self.packed = packed
        self.want_script = want_script
        flags = (SED_WANT_SCRIPT if want_script else (SED_NO_LEN if no_len else 0)) | \
            (SED_PIPELINE if pipeline else 0)
        self.ptr = self._lib.sed_batch_create(ctx.ptr, packed.codes_a, packed.off_a, packed.len_a, packed.codes_b,
                                              packed.off_b, packed.len_b, packed.npairs, flags)
        if not self.ptr:
            msg = self._lib.sed_last_error(ctx.ptr)
            raise SedError("sed_batch_create failed: %s" % (msg.decode() if msg else ""))

    def close(self):
        if self.ptr:
            self._lib.sed_batch_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def mode(self):
        return MODE_NAMES.get(self._lib.sed_batch_mode(self.ptr), "?")

    @property
    def rows_per_lane(self):
        return self._lib.sed_batch_rows_per_lane(self.ptr)

    @property
    def lane_pairs(self):
        return self._lib.sed_batch_lane_pairs(self.ptr)

    @property
    def chains(self):
        return self._lib.sed_batch_chains(self.ptr)

    @property
    def traceback_mode(self):
        """0 distance only, 1 per-cell traceback codes, 2 checkpoints + recompute (SED_OPT_TB)."""
        return self._lib.sed_batch_traceback_mode(self.ptr)

    def chain_stats(self):
        """(pairs handed out by the dynamic-CHAIN counter, most pairs one wave computed) of the last run."""
        f, mx = C.c_int32(), C.c_int32()
        self.ctx._check(self._lib.sed_batch_chain_stats(self.ptr, C.byref(f), C.byref(mx)), "sed_batch_chain_stats")
        return f.value, mx.value

    @property
    def packed_pairs(self):
        """Pairs computed two per lane / per wave in packed 16-bit cells (distance-only batches)."""
        return self._lib.sed_batch_packed_pairs(self.ptr)

    def run(self):
        self.ctx._check(self._lib.sed_batch_run(self.ptr), "sed_batch_run")

    def sync(self):
        self.ctx._check(self._lib.sed_batch_sync(self.ptr), "sed_batch_sync")

    def last_times(self):
        a, b = C.c_float(), C.c_float()
        self.ctx._check(self._lib.sed_batch_last_times(self.ptr, C.byref(a), C.byref(b)), "sed_batch_last_times")
        return a.value, b.value

    def times(self, max_runs=4096):
        """(dp_ms[], traceback_ms[]) of every run since reset_times(), from HIP events."""
        a = np.zeros(max_runs, np.float32)
        b = np.zeros(max_runs, np.float32)
        cnt = self._lib.sed_batch_times(self.ptr, a, b, max_runs)
        if cnt < 0:
            self.ctx._check(cnt, "sed_batch_times")
        return a[:cnt].astype(np.float64), b[:cnt].astype(np.float64)

    def reset_times(self):
        self._lib.sed_batch_reset_times(self.ptr)

    def work(self):
        a, b = C.c_double(), C.c_double()
        self._lib.sed_batch_work(self.ptr, C.byref(a), C.byref(b))
        return a.value, b.value

    def device_results(self):
        vals = [C.c_uint64() for _ in range(5)]
        self._lib.sed_batch_device_results(self.ptr, *[C.byref(v) for v in vals])
        return [v.value for v in vals]

    def export(self, d_dist=0, d_len=0, d_ops=0):
        """Device-to-device copy of the results into caller memory (raw device pointers)."""
        self.ctx._check(self._lib.sed_batch_export(self.ptr, d_dist, d_len, d_ops), "sed_batch_export")

    def results(self):
        P = self.packed.npairs
        dist = np.zeros(max(P, 1), np.float64)
        is_int = np.zeros(max(P, 1), np.uint8)
        ln = np.zeros(max(P, 1), np.int32)
        ops = None
        ops_ptr = off_ptr = None
        if self.want_script:
            ops = np.zeros(max(int(self.packed.ops_off[P]), 1), np.uint32)
            ops_ptr = ops.ctypes.data_as(C.c_void_p)
            off_ptr = self.packed.ops_off.ctypes.data_as(C.c_void_p)
        self.ctx._check(self._lib.sed_batch_results(self.ptr, dist, is_int, ln, ops_ptr, off_ptr), "sed_batch_results")
        return dist[:P], is_int[:P], ln[:P], ops


_ctx = None


def context(device=None):
    """Process-wide default context (device from SED_DEVICE / LOCAL_RANK, else 0)."""
    global _ctx
    with _lock:
        if _ctx is None:
            if device is None:
                device = int(os.environ.get("SED_DEVICE", os.environ.get("LOCAL_RANK", "0")))
            _ctx = Context(device)
        return _ctx
