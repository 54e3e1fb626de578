"""ctypes binding of libsed.so (include/sed.h) — the only way the Python side
reaches the GPU engine.  There is deliberately no CPU fallback: if the library
or a HIP device is missing, every entry point raises.

Process model.  The reference's callers parallelise by forking: gui.py runs
wagnerFisher in the GUI process (gui.py:360), then IRMethods.create_search_threads
forks a multiprocessing.Process per similarity method and again for wf_score
(IRMethods.py:487-491, 511-514).  HIP cannot be used in a child forked after the
parent initialised it.  context() therefore returns, in such a child, an
EngineClient that sends every call to an engine that owns a HIP context:
  - by default the parent itself: every fork of a process that holds a Context
    gets a socket pair.  One selector thread of the parent watches the pairs;
    a child's first request starts a thread that serves it on a Context of its
    own (from a pool of two, else a new one), and children that never call the
    engine cost only their socket.  A child pays no start-up beyond that
    sed_create, which is what create_search_threads' two Process rounds need.
    Served children need the parent alive: when it exits, their calls raise;
  - otherwise (SED_FORK_ENGINE=worker, a grandchild, or a fork taken while no
    Context existed) the child starts one engine worker, a fresh interpreter
    running this file, and talks to it over a pipe pair.
Processes that never inherited a HIP context use the GPU directly.
SED_ENGINE=worker keeps HIP out of the calling process always; SED_ENGINE=inproc
forbids both (a forked child then raises SedError).  An inherited Context is
never touched by the child (not even by __del__).
"""
import ctypes as C
import os
import pickle
import socket
import subprocess
import sys
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
SED_OPT_DOT = 10
SED_OPT_BITPAR = 11
SED_OPT_SCALED = 12
SED_OPT_SEG = 13
SED_OPT_SPLITCK = 14
SED_OPT_ZEROCOPY = 15
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
    ("sed_batch_dot_keys", C.c_int, [C.c_void_p]),
    ("sed_dot_factor", C.c_int, [_f64p, C.c_double, C.c_double, C.c_int, C.c_int, _u32p]),
    ("sed_batch_packed_pairs", C.c_int, [C.c_void_p]),
    ("sed_batch_bitpar_pairs", C.c_int, [C.c_void_p]),
    ("sed_batch_scaled_pairs", C.c_int, [C.c_void_p]),
    ("sed_batch_segment_pairs", C.c_int, [C.c_void_p]),
    ("sed_batch_split_tasks", C.c_int, [C.c_void_p]),
    ("sed_batch_traceback_mode", C.c_int, [C.c_void_p]),
    ("sed_batch_chain_stats", C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("sed_batch_run", C.c_int, [C.c_void_p]),
    ("sed_batch_sync", C.c_int, [C.c_void_p]),
    ("sed_batch_last_times", C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    ("sed_batch_times", C.c_int, [C.c_void_p, _f32p, _f32p, C.c_int]),
    ("sed_batch_spans", C.c_int, [C.c_void_p, _f32p, C.c_int]),
    ("sed_batch_reset_times", C.c_int, [C.c_void_p]),
    ("sed_batch_set_timing", C.c_int, [C.c_void_p, C.c_int]),
    ("sed_run_pair", C.c_int, [C.c_void_p, C.c_char_p, C.c_int32, C.c_char_p, C.c_int32, C.c_uint32, C.c_void_p,
                               C.c_void_p, C.c_void_p, C.c_void_p]),
    ("sed_pair_submit", C.c_int, [C.c_void_p, C.c_char_p, C.c_int32, C.c_char_p, C.c_int32, C.c_uint32]),
    ("sed_pair_wait", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("sed_batch_results", C.c_int, [C.c_void_p, _f64p, _u8p, _i32p, C.c_void_p, C.c_void_p]),
    ("sed_batch_dp_launches", C.c_int, [C.c_void_p]),
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


_hip_pid = None  # pid of the process whose HIP context this module created (inherited by forked children)


class Context:
    """One sed_ctx (device + stream + cost table), owned by the process that created it."""

    def __init__(self, device=0):
        global _hip_pid
        if _hip_pid is not None and _hip_pid != os.getpid():
            raise SedError("HIP was initialised by process %d and this process is a fork of it: use "
                           "sedgpu.context(), which runs the engine in a worker process" % _hip_pid)
        lib = load()
        self._lib = lib
        self._pid = os.getpid()
        self.device = device
        self.ptr = lib.sed_create(device)
        _hip_pid = self._pid
        if not self.ptr:
            raise SedError("sed_create(%d) failed: no usable HIP device" % device)
        self._cost_key = None
        self._cost_plan = None
        self._pair_out = None
        self._pending = None  # (want_script, script words) of a submit_pair not yet waited for

    def close(self):
        # a forked child must not call into the parent's HIP context (it would destroy or hang on it)
        if self.ptr and self._pid == os.getpid():
            self._lib.sed_destroy(self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if self._pid != os.getpid():
            raise SedError("%s: this Context belongs to process %d (fork); use sedgpu.context()" % (what, self._pid))
        if rc != 0:
            msg = self._lib.sed_last_error(self.ptr)
            raise SedError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))

    def set_option(self, key, value):
        self._check(self._lib.sed_set_option(self.ptr, key, value), "sed_set_option")

    def set_mode(self, mode):
        """0 auto, 1 integer, 2 fp64, 3 fp64 with int typing."""
        self.set_option(SED_OPT_MODE, mode)
        self.invalidate_costs()

    def invalidate_costs(self):
        """Forget the cached cost plan: the next set_costs() uploads its table.  Call it after any direct
        lib.sed_set_costs / mode change that bypasses set_costs()."""
        self._cost_key = None
        self._cost_plan = None

    def set_costs(self, plan):
        if plan is self._cost_plan:  # (sedcost.pair_plan hands out the same plan object for the same costs)
            return
        key = plan.key()
        if key == self._cost_key:
            self._cost_plan = plan
            return
        self._cost_plan = None
        sub = np.ascontiguousarray(plan.sub, dtype=np.float64).ravel()
        sub_int = np.ascontiguousarray(plan.sub_int, dtype=np.uint8).ravel()
        self._check(self._lib.sed_set_costs(self.ptr, plan.K, sub, sub_int, plan.ins, plan.ins_int,
                                            plan.dele, plan.del_int), "sed_set_costs")
        self._cost_key = key
        self._cost_plan = plan

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

    def run_pair(self, codes_a, codes_b, want_script, no_len=False):
        """One pair (codes as bytes): (dist, is_int, len, ops u32[] | None) through sed_run_pair, the per-call path of
        the drop-in module (no numpy arrays on the way in, preallocated result cells on the way out)."""
        if self._pid != os.getpid():
            self._check(0, "sed_run_pair")
        r = self._pair_out
        if r is None:
            r = self._pair_out = (C.c_double(), C.c_uint8(), C.c_int32())
        ops = None
        ops_ptr = None
        if want_script:
            ops = np.zeros(max(1, (len(codes_a) + len(codes_b) + 15) // 16), np.uint32)
            ops_ptr = ops.ctypes.data
        flags = SED_WANT_SCRIPT if want_script else (SED_NO_LEN if no_len else 0)
        rc = self._lib.sed_run_pair(self.ptr, codes_a, len(codes_a), codes_b, len(codes_b), flags, C.addressof(r[0]),
                                    C.addressof(r[1]), C.addressof(r[2]), ops_ptr)
        if rc != 0:
            self._check(rc, "sed_run_pair")
        return r[0].value, r[1].value, r[2].value, ops

    def submit_pair(self, codes_a, codes_b, want_script, no_len=False):
        """run_pair's first half (sed_pair_submit): the pair's kernels are enqueued and this returns at once;
        wait_pair() returns what run_pair would have."""
        if self._pid != os.getpid():
            self._check(0, "sed_pair_submit")
        flags = SED_WANT_SCRIPT if want_script else (SED_NO_LEN if no_len else 0)
        rc = self._lib.sed_pair_submit(self.ptr, codes_a, len(codes_a), codes_b, len(codes_b), flags)
        if rc != 0:
            self._check(rc, "sed_pair_submit")
        self._pending = (want_script, (len(codes_a) + len(codes_b) + 15) // 16)

    def wait_pair(self):
        """(dist, is_int, len, ops u32[] | None) of the pair submit_pair enqueued (sed_pair_wait)."""
        want_script, words = self._pending
        self._pending = None
        r = self._pair_out
        if r is None:
            r = self._pair_out = (C.c_double(), C.c_uint8(), C.c_int32())
        ops = np.zeros(max(1, words), np.uint32) if want_script else None
        rc = self._lib.sed_pair_wait(self.ptr, C.addressof(r[0]), C.addressof(r[1]), C.addressof(r[2]),
                                     ops.ctypes.data if want_script else None)
        if rc != 0:
            self._check(rc, "sed_pair_wait")
        return r[0].value, r[1].value, r[2].value, ops

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
    def from_concat(cls, codes_a, len_a, codes_b, len_b):
        """Pairs from concatenated codes and per-pair lengths (CostPlan.encode_many)."""
        self = cls.__new__(cls)
        P = len(len_a)
        self.npairs = P
        self.len_a = np.asarray(len_a, np.int32) if P else np.zeros(1, np.int32)
        self.len_b = np.asarray(len_b, np.int32) if P else np.zeros(1, np.int32)
        self.off_a = np.zeros(max(P, 1), np.int64)
        self.off_b = np.zeros(max(P, 1), np.int64)
        if P:
            self.off_a[1:] = np.cumsum(self.len_a[:-1])
            self.off_b[1:] = np.cumsum(self.len_b[:-1])
        self.codes_a = np.concatenate([np.asarray(codes_a, np.uint8), np.zeros(1, np.uint8)])
        self.codes_b = np.concatenate([np.asarray(codes_b, np.uint8), np.zeros(1, np.uint8)])
        words = (self.len_a.astype(np.int64) + self.len_b + 15) // 16
        self.ops_off = np.zeros(max(P, 1) + 1, np.int64)
        if P:
            self.ops_off[1:P + 1] = np.cumsum(words[:P])
        return self

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
        if self.ptr and self.ctx._pid == os.getpid():
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
    def dot_keys(self):
        """True when the checkpoint forward kernel runs dot keys (v_dot4 + v_max3 per cell, SED_OPT_DOT)."""
        return (self._lib.sed_batch_dot_keys(self.ptr) & 1) == 1

    @property
    def ladder_dot_keys(self):
        """True when the CHAIN kernel runs ladder keys with the update addend as one v_dot4 (SED_OPT_DOT)."""
        return (self._lib.sed_batch_dot_keys(self.ptr) & 2) == 2

    @property
    def ladder_wide(self):
        """True when those ladder dot keys run over the wide ladder (V = D*A + 16L, one jump row in 8)."""
        return (self._lib.sed_batch_dot_keys(self.ptr) & 4) == 4

    @property
    def traceback_mode(self):
        """0 distance only, 1 per-cell traceback codes, 2 checkpoints + recompute (SED_OPT_TB), 3 per-cell codes walked
        stripe-parallel, 4 SPLIT checkpoints recomputed into per-cell codes (SED_OPT_SPLITCK)."""
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

    @property
    def bitpar_pairs(self):
        """Lane pairs computed bit-parallel (unit costs, distance only; SED_OPT_BITPAR)."""
        return self._lib.sed_batch_bitpar_pairs(self.ptr)

    @property
    def scaled_pairs(self):
        """fp64 lane pairs computed as an exact integer DP of costs scaled by 2^k (dyadic tables, SED_OPT_SCALED)."""
        return self._lib.sed_batch_scaled_pairs(self.ptr)

    @property
    def segment_pairs(self):
        """fp64 wave pairs computed in 16-lane segments, four per wave (SED_OPT_SEG)."""
        return self._lib.sed_batch_segment_pairs(self.ptr)

    @property
    def split_tasks(self):
        """SPLIT batches: the (pair, stripe) workgroups of a run, 0 otherwise (SED_OPT_SPLIT)."""
        return self._lib.sed_batch_split_tasks(self.ptr)

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

    def spans(self, max_runs=4096):
        """Every run since reset_times() as intervals: array [runs, parts, 4] of {DP start, DP end, traceback start,
        traceback end} in ms from the first run's DP start (HIP events on the launching streams)."""
        P = max(1, self.dp_launches)
        out = np.zeros(max_runs * P * 4, np.float32)
        cnt = self._lib.sed_batch_spans(self.ptr, out, max_runs)
        if cnt < 0:
            self.ctx._check(cnt, "sed_batch_spans")
        return out[:cnt * P * 4].reshape(cnt, P, 4).astype(np.float64)

    def reset_times(self):
        self._lib.sed_batch_reset_times(self.ptr)

    def set_timing(self, every):
        """Timing events on every run (1), every k-th run (k), or none (0)."""
        self.ctx._check(self._lib.sed_batch_set_timing(self.ptr, int(every)), "sed_batch_set_timing")

    def work(self):
        a, b = C.c_double(), C.c_double()
        self._lib.sed_batch_work(self.ptr, C.byref(a), C.byref(b))
        return a.value, b.value

    @property
    def dp_launches(self):
        """Forward launches per run: a checkpoint batch of >= 2048 wave pairs runs in parts on as many streams
        (SED_CK_HALVES, default 2), else 1.  With parts, times() and last_times() are the mean launch over the parts
        (which overlap each other's kernels); spans() gives every part's intervals."""
        return self._lib.sed_batch_dp_launches(self.ptr)

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


class EngineClient:
    """The Context interface (set_costs, set_option, set_mode, run, full_matrix, selftest) served by an
    engine worker process: a fresh interpreter running this file, started on first use, that owns its
    own HIP context.  One request at a time over a pipe pair; the worker exits when the pipe closes."""

    def __init__(self, device=0, channel=None):
        self.device = device
        self._proc = None
        self._tx = self._rx = None
        self._cost_key = None
        self._pid = os.getpid()
        self._channel = channel  # this process's socket to its parent's engine thread (None: start a worker)
        self.served_by = None

    def _start(self):
        from multiprocessing.connection import Connection
        if self._channel is not None:  # the parent serves this child (see the module docstring)
            sock, self._channel = self._channel, None
            self._tx = self._rx = Connection(sock.detach())
            self.served_by = "parent"
            self._tx.send_bytes(pickle.dumps(("open", self.device), protocol=pickle.HIGHEST_PROTOCOL))
            status, val = pickle.loads(self._rx.recv_bytes())
            if status != "ok":
                raise SedError(val)
            return
        self.served_by = "worker"
        c2w_r, c2w_w = os.pipe()
        w2c_r, w2c_w = os.pipe()
        env = dict(os.environ)
        env["SED_ENGINE"] = "inproc"
        try:
            self._proc = subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), "--engine-worker",
                                           str(self.device), str(c2w_r), str(w2c_w)],
                                          pass_fds=(c2w_r, w2c_w), close_fds=True, env=env)
        finally:
            os.close(c2w_r)
            os.close(w2c_w)
        self._tx = Connection(c2w_w, readable=False)
        self._rx = Connection(w2c_r, writable=False)

    def _call(self, *req):
        if self._pid != os.getpid():  # a fork of a process with a client: start its own worker
            self.__init__(self.device)
        if self._tx is None:
            self._start()
        try:
            self._tx.send_bytes(pickle.dumps(req, protocol=pickle.HIGHEST_PROTOCOL))
            status, val = pickle.loads(self._rx.recv_bytes())
        except (EOFError, OSError) as ex:
            raise SedError("engine worker (pid %s) is gone: %s" % (self._proc.pid if self._proc else "?", ex))
        if status != "ok":
            raise SedError(val)
        return val

    def close(self):
        if self._tx is not None and self._pid == os.getpid():
            for f in {id(self._tx): self._tx, id(self._rx): self._rx}.values():
                try:
                    f.close()
                except OSError:
                    pass
            if self._proc is not None:
                try:
                    self._proc.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    self._proc.kill()
        self._proc = None
        self._tx = self._rx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, key, value):
        self._call("set_option", key, value)

    def set_mode(self, mode):
        self.set_option(SED_OPT_MODE, mode)
        self.invalidate_costs()

    def invalidate_costs(self):
        self._cost_key = None

    def set_costs(self, plan):
        key = plan.key()
        if key == self._cost_key:
            return
        self._call("set_costs", plan.K, plan.sub, plan.sub_int, plan.ins, plan.ins_int, plan.dele, plan.del_int)
        self._cost_key = key

    def selftest(self):
        return self._call("selftest")

    def run(self, packed, want_script, no_len=False):
        return self._call("run", packed, want_script, no_len)

    def run_pair(self, codes_a, codes_b, want_script, no_len=False):
        return self._call("run_pair", codes_a, codes_b, want_script, no_len)

    def full_matrix(self, codes_a, codes_b):
        return self._call("full_matrix", np.asarray(codes_a, np.uint8), np.asarray(codes_b, np.uint8))


class _PlanArgs:
    """The fields Context.set_costs reads from a sedcost.CostPlan."""

    def __init__(self, K, sub, sub_int, ins, ins_int, dele, del_int):
        self.K, self.sub, self.sub_int = K, sub, sub_int
        self.ins, self.ins_int, self.dele, self.del_int = ins, ins_int, dele, del_int

    def key(self):
        return (self.K, self.sub.tobytes(), self.sub_int.tobytes(), self.ins, self.ins_int, self.dele, self.del_int)


_serve_pool = []  # idle serving Contexts of this process (parent-served children): the next child reuses one
_serve_pool_lock = threading.Lock()


def _serve(rx, tx, device, pooled=False):
    """Serve EngineClient requests on one Context until the client closes its end.  pooled: the Context comes from
    and returns to _serve_pool (a parent serving its forked children: create_search_threads' second Process then
    starts without a sed_create), with the options the client set put back to their defaults."""
    ctx = None
    touched = set()
    while True:
        try:
            req = pickle.loads(rx.recv_bytes())
        except (EOFError, OSError):
            break
        try:
            op, args = req[0], req[1:]
            if op == "open":  # (a parent-served child names its device first)
                device = args[0]
            if ctx is None:
                if pooled:
                    with _serve_pool_lock:
                        for x in _serve_pool:
                            if x.device == device:
                                _serve_pool.remove(x)
                                ctx = x
                                break
                if ctx is None:
                    ctx = Context(device)
            if op == "open":
                val = None
            elif op == "set_costs":
                ctx.set_costs(_PlanArgs(*args))
                val = None
            elif op == "set_option":
                ctx.set_option(*args)
                touched.add(args[0])
                val = None
            elif op == "selftest":
                val = ctx.selftest()
            elif op == "run":
                val = ctx.run(*args)
            elif op == "run_pair":
                val = ctx.run_pair(*args)
            elif op == "full_matrix":
                val = ctx.full_matrix(*args)
            else:
                raise SedError("unknown engine request %r" % (op,))
            out = ("ok", val)
        except Exception as ex:  # reported to the client as SedError
            out = ("err", "%s: %s" % (type(ex).__name__, ex))
        try:
            tx.send_bytes(pickle.dumps(out, protocol=pickle.HIGHEST_PROTOCOL))
        except OSError:
            break
    if ctx is not None and pooled:
        try:
            for key in touched:
                ctx.set_option(key, 0)
            if touched:
                ctx.invalidate_costs()
            with _serve_pool_lock:
                if len(_serve_pool) < 2:
                    _serve_pool.append(ctx)
                    ctx = None
        except SedError:
            pass
    if ctx is not None:
        ctx.close()


def _engine_worker(device, rfd, wfd):
    """The worker process's main loop."""
    from multiprocessing.connection import Connection
    _serve(Connection(rfd, writable=False), Connection(wfd, readable=False), device)


def _serve_child(sock):
    """Thread of a HIP process serving one forked child over its socket pair."""
    from multiprocessing.connection import Connection
    conn = Connection(sock.detach())
    try:
        _serve(conn, conn, 0, pooled=True)
    finally:
        conn.close()


# fork hooks: a process holding a HIP Context gives each fork a socket pair.  The parent's ends are watched by one
# selector thread (started at the first fork); a child's first request starts a thread serving that child, and a child
# that exits without using the engine (a Manager server, a helper) only has its socket closed.  Served children depend
# on this process: when it exits, their channels close and their next engine call raises SedError.
_fork_pair = None
_child_channel = None  # (socket, pid) in a child forked from a HIP process
_sel_state = None  # parent: (selector, wake read end, wake write end, channels to register)
_sel_lock = threading.Lock()


def _watch_channel(sock):
    """Hand the parent's end of a new child's socket pair to the selector thread."""
    global _sel_state
    with _sel_lock:
        if _sel_state is None:
            import selectors
            sel = selectors.DefaultSelector()
            wr, ww = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
            wr.setblocking(False)
            sel.register(wr, selectors.EVENT_READ)
            _sel_state = (sel, wr, ww, [])
            threading.Thread(target=_channel_selector, args=(_sel_state,), daemon=True,
                             name="sed-engine-channels").start()
        _sel_state[3].append(sock)
        ww = _sel_state[2]
    ww.send(b"\0")


def _channel_selector(state):
    """The selector thread: waits on every child's channel until its first request (or its end)."""
    import selectors
    sel, wake, _, pending = state
    while True:
        for key, _ in sel.select():
            s = key.fileobj
            if s is wake:
                try:
                    wake.recv(4096)
                except BlockingIOError:
                    pass
                with _sel_lock:
                    new, pending[:] = list(pending), []
                for x in new:
                    sel.register(x, selectors.EVENT_READ)
                continue
            sel.unregister(s)
            try:
                first = s.recv(1, socket.MSG_PEEK)
            except OSError:
                first = b""
            if first:
                threading.Thread(target=_serve_child, args=(s,), daemon=True, name="sed-engine-fork").start()
            else:
                s.close()  # the child closed its end without a request


def _before_fork():
    global _fork_pair
    _fork_pair = None
    if _hip_pid == os.getpid() and os.environ.get("SED_FORK_ENGINE", "parent") == "parent":
        try:
            _fork_pair = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
        except OSError:
            _fork_pair = None


def _after_fork_in_parent():
    global _fork_pair
    pair, _fork_pair = _fork_pair, None
    if pair is not None:
        pair[1].close()
        _watch_channel(pair[0])


_ctx = None
_ctx_pid = None


def _reset_lock_in_child():
    global _lock, _fork_pair, _child_channel, _sel_state, _sel_lock
    _lock = threading.Lock()  # a fork taken while another thread held it must not deadlock the child
    _sel_lock = threading.Lock()
    st, _sel_state = _sel_state, None  # (the parent's selector thread does not exist here: drop its copies)
    if st is not None:
        for x in (st[0], st[1], st[2]):
            try:
                x.close()
            except OSError:
                pass
    if _child_channel is not None and _child_channel[1] != os.getpid():
        # a channel this process's parent got but never used: a grandchild must not hold it open
        try:
            _child_channel[0].close()
        except OSError:
            pass
    pair, _fork_pair = _fork_pair, None
    if pair is not None:
        pair[0].close()
        _child_channel = (pair[1], os.getpid())
    else:
        _child_channel = None


if hasattr(os, "register_at_fork"):
    os.register_at_fork(before=_before_fork, after_in_parent=_after_fork_in_parent, after_in_child=_reset_lock_in_child)


def context(device=None):
    """Process-wide default engine (device from SED_DEVICE / LOCAL_RANK, else 0): an in-process Context,
    or an EngineClient in a child forked after its parent initialised HIP (or with SED_ENGINE=worker)."""
    global _ctx, _ctx_pid, _child_channel
    with _lock:
        pid = os.getpid()
        if _ctx is None or _ctx_pid != pid:
            if device is None:
                device = int(os.environ.get("SED_DEVICE", os.environ.get("LOCAL_RANK", "0")))
            mode = os.environ.get("SED_ENGINE", "auto")
            inherited = _hip_pid is not None and _hip_pid != pid
            if mode == "worker" or (inherited and mode != "inproc"):
                ch = _child_channel[0] if (_child_channel and _child_channel[1] == pid and mode != "worker") else None
                _child_channel = None  # (one client per channel)
                _ctx = EngineClient(device, ch)
            else:
                _ctx = Context(device)  # raises SedError in a fork of a HIP process (SED_ENGINE=inproc)
            _ctx_pid = pid
        return _ctx


if __name__ == "__main__" and len(sys.argv) == 5 and sys.argv[1] == "--engine-worker":
    _engine_worker(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))


def dot_factor(sub, ins, dele, maxmin=0, ladder_maxsum=0):
    """The byte factorisation behind SED_OPT_DOT (no device needed): (A, rows, cols, aux) or None.
    sub: 4 x 4 costs (row symbol -> column symbol); rows/cols: 4 x 4 signed bytes; aux = (decode shift, multiplier),
    or for the ladder keys (ladder_maxsum > 0) (sentinel byte, L unit: 16 on the wide ladder, else 8)."""
    out = np.zeros(10, np.uint32)
    A = load().sed_dot_factor(np.ascontiguousarray(sub, np.float64).ravel(), float(ins), float(dele), int(maxmin),
                              int(ladder_maxsum), out)
    if A < 0:
        raise SedError("sed_dot_factor: bad arguments")
    if A == 0:
        return None
    to_bytes = lambda w: np.frombuffer(np.asarray(w, np.uint32).tobytes(), np.int8).reshape(4, 4).astype(np.int64)
    return A, to_bytes(out[0:4]), to_bytes(out[4:8]), (int(out[8]), int(out[9]))
