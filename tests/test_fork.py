"""CPU: the drop-in module under the reference's process model (IRMethods.create_search_threads forks a
multiprocessing.Process per method after gui.py ran wagnerFisher in the parent, IRMethods.py:487-491,
511-514).  A child forked after its parent initialised HIP must never call into the inherited context:
sedgpu.context() gives it an EngineClient served by a thread of the parent on a Context of its own (or, with
SED_FORK_ENGINE=worker, by an engine worker process; SED_ENGINE=inproc: a clear SedError).  Here the parent's
HIP initialisation is simulated (no GPU in this container), so the serving Context itself reports that no
device exists -- as an error, within seconds, not a hang."""
import multiprocessing as mp
import os

import numpy as np
import pytest

import sedgpu


class _NoCallLib:
    """Stands in for libsed in an inherited Context: any call from the child fails the test."""

    def __getattr__(self, name):
        raise AssertionError("child called %s on the parent's HIP context" % name)


def _child(q, engine, fork_engine=None):
    try:
        if engine is not None:
            os.environ["SED_ENGINE"] = engine
        if fork_engine is not None:
            os.environ["SED_FORK_ENGINE"] = fork_engine
        inherited = sedgpu._ctx
        inherited.close()  # must not touch the parent's context
        assert inherited.ptr is None
        ctx = sedgpu.context()
        kind = type(ctx).__name__
        packed = sedgpu.PackedPairs([np.array([0, 1, 2], np.uint8)], [np.array([0, 2], np.uint8)])
        try:
            ctx.run(packed, False)
            q.put((kind, "no error", ctx.served_by))
        except sedgpu.SedError as ex:
            q.put((kind, str(ex), ctx.served_by))
    except BaseException as ex:  # reported to the parent
        q.put(("crash", repr(ex), None))


def _fake_parent_context():
    """A Context as the parent would hold after gui.py's wagnerFisher (HIP initialised in this pid)."""
    c = sedgpu.Context.__new__(sedgpu.Context)
    c._lib, c.ptr, c._pid, c._cost_key = _NoCallLib(), 12345, os.getpid(), None
    return c


@pytest.mark.parametrize("engine,fork_engine", [(None, None), (None, "worker"), ("inproc", None)])
def test_forked_child_never_uses_the_parents_hip_context(monkeypatch, engine, fork_engine):
    """Default: the parent serves the child on a Context of its own (a thread per fork, over a socket pair);
    SED_FORK_ENGINE=worker: the child starts an engine worker; SED_ENGINE=inproc: the child raises."""
    monkeypatch.setattr(sedgpu, "_hip_pid", os.getpid())
    monkeypatch.setattr(sedgpu, "_ctx", _fake_parent_context())
    monkeypatch.setattr(sedgpu, "_ctx_pid", os.getpid())
    monkeypatch.delenv("SED_ENGINE", raising=False)
    monkeypatch.delenv("SED_FORK_ENGINE", raising=False)
    if fork_engine:
        monkeypatch.setenv("SED_FORK_ENGINE", fork_engine)  # (read by the parent's fork hook too)
    fork = mp.get_context("fork")
    q = fork.Queue()
    p = fork.Process(target=_child, args=(q, engine, fork_engine))
    p.start()
    kind, msg, served = q.get(timeout=120)
    p.join(timeout=60)
    assert p.exitcode == 0
    if engine == "inproc":
        assert kind == "crash" and "fork" in msg  # context() refuses to build a Context in the fork
    else:
        assert kind == "EngineClient", msg
        assert served == (fork_engine or "parent")
        # no device here: the serving Context (the parent's thread, or the worker) reports it as SedError
        assert "sed_create(0) failed" in msg or "libsed.so not found" in msg, msg
    sedgpu._ctx.ptr = None  # the fake must not reach sed_destroy here either


def test_worker_engine_reports_errors_without_a_device(monkeypatch):
    """SED_ENGINE=worker: the calling process never loads HIP; requests go to the worker, whose errors
    come back as SedError."""
    monkeypatch.setattr(sedgpu, "_ctx", None)
    monkeypatch.setattr(sedgpu, "_ctx_pid", None)
    monkeypatch.setenv("SED_ENGINE", "worker")
    ctx = sedgpu.context()
    assert isinstance(ctx, sedgpu.EngineClient)
    with pytest.raises(sedgpu.SedError):
        ctx.selftest()
    ctx.close()
    monkeypatch.setattr(sedgpu, "_ctx", None)


def _idle_child():
    pass  # forked, never touches the engine


def _grandchild_probe(q):
    """In a forked child that holds an unused channel: fork a grandchild, which must hold neither the channel object
    nor its descriptor."""
    fd = sedgpu._child_channel[0].fileno() if sedgpu._child_channel else -1
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:
        ok = sedgpu._child_channel is None
        try:
            os.fstat(fd)
            ok = False  # still open in the grandchild
        except OSError:
            pass
        os.write(w, b"1" if ok else b"0")
        os._exit(0)
    os.waitpid(pid, 0)
    q.put((fd, os.read(r, 1)))


def test_fork_channels_share_one_selector_thread(monkeypatch):
    """Forks of a HIP process get channels watched by one selector thread: children that never use the engine get
    no serving thread (their channels are closed when they exit), and a child's unused channel is closed in its own
    forks."""
    import threading
    import time
    monkeypatch.setattr(sedgpu, "_hip_pid", os.getpid())
    monkeypatch.setattr(sedgpu, "_ctx", _fake_parent_context())
    monkeypatch.setattr(sedgpu, "_ctx_pid", os.getpid())
    monkeypatch.delenv("SED_FORK_ENGINE", raising=False)
    serving = lambda: sum(t.name == "sed-engine-fork" for t in threading.enumerate())
    before = serving()
    fork = mp.get_context("fork")
    procs = [fork.Process(target=_idle_child) for _ in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    q = fork.Queue()
    p = fork.Process(target=_grandchild_probe, args=(q,))
    p.start()
    fd, ok = q.get(timeout=60)
    p.join(timeout=60)
    assert fd >= 0 and ok == b"1"
    time.sleep(0.3)
    names = [t.name for t in threading.enumerate()]
    assert names.count("sed-engine-channels") == 1
    assert serving() <= before  # no child made a request
    sedgpu._ctx.ptr = None
