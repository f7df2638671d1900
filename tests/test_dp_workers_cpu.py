"""DataParallel's per-device replay workers (parallel/dp.py run_workers): one host thread per
device enqueues that device's graph segment; a worker that raises, or that never returns, must
surface in the training step as an exception within a bounded time -- never a hang."""
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import pytest

from pytorch_distributed_amd.parallel.dp import run_workers


def test_results_in_order():
    with ThreadPoolExecutor(4) as pool:
        assert run_workers(pool, [lambda i=i: i * i for i in range(4)], 5.0) == [0, 1, 4, 9]


def test_worker_exception_names_device():
    def bad():
        time.sleep(0.05)
        raise ValueError("injected replay failure")
    with ThreadPoolExecutor(3) as pool:
        t0 = time.time()
        with pytest.raises(RuntimeError, match=r"cuda:1 failed: ValueError: injected replay failure"):
            run_workers(pool, [lambda: 0, bad, lambda: 2], 30.0, ["cuda:0", "cuda:1", "cuda:2"])
        assert time.time() - t0 < 5.0


def test_hung_worker_times_out():
    stop = threading.Event()
    with ThreadPoolExecutor(2) as pool:
        t0 = time.time()
        with pytest.raises(TimeoutError, match=r"cuda:1"):
            run_workers(pool, [lambda: 0, lambda: stop.wait(60)], 0.5, ["cuda:0", "cuda:1"])
        assert time.time() - t0 < 5.0
        stop.set()


class _FakeStream:
    def __init__(self, log, name):
        self.log, self.name = log, name

    def wait_stream(self, other):
        self.log.append(("wait", self.name, other.name))


class _FakeDev:
    def __init__(self, i):
        self.index = i


class _FakeReplica:
    """A replica graph with ``nseg`` segments whose all-reduce points are ``ends``."""

    def __init__(self, i, nseg, ends, log):
        self.dev = _FakeDev(i)
        self.graphs = [object()] * nseg
        self.seg_reduce = ends
        self.side_split = False
        self.log = log
        self.i = i

    def replay(self, s, x, y, st):
        self.log.append(("replay", self.i, s, threading.current_thread().name))

    def replay_range(self, s0, s1, x, y, st):
        for s in range(s0, s1 + 1):
            self.replay(s, x, y, st)

    def join_side(self, st):
        pass


@pytest.mark.parametrize("threaded", [True, False])
def test_overlapped_replay_order_and_reduce_points(threaded, monkeypatch):
    """_replay_overlapped over fake replicas: every replica replays every segment once, in order;
    each gradient slice is all-reduced after every replica has enqueued the segments that complete
    it, slices in order; the threaded path hands each device ONE task per reduce interval (the ~65
    segments of a per-weight-gradient capture would otherwise cost a pool round trip each)."""
    from pytorch_distributed_amd.parallel import dp as dpmod
    monkeypatch.setenv("PDA_DP_THREADS", "1" if threaded else "0")
    log = []
    nseg, ends = 9, [None, None, 10, None, 20, None, None, None, 30]
    calls = []
    real = dpmod.run_workers
    monkeypatch.setattr(dpmod, "run_workers",
                        lambda pool, fns, t, names=None: calls.append(len(fns)) or real(pool, fns, t, names))
    class _DP(dpmod.DataParallel):
        all_modules = property(lambda self: [])
    obj = _DP.__new__(_DP)
    dpmod.nn.Module.__init__(obj)
    obj.device_ids = [0, 1, 2]
    obj.timing = False
    obj.replay_timeout_s = 30.0
    cs = [_FakeStream(log, f"comm{i}") for i in range(3)]
    obj._comm_streams = lambda: cs
    obj._reduce_slice = lambda lo, hi, streams=None: log.append(("reduce", lo, hi))
    pool = ThreadPoolExecutor(3)
    obj._pool = lambda: pool
    jobs = [(_FakeReplica(i, nseg, ends, log), None, None) for i in range(3)]
    streams = [_FakeStream(log, f"main{i}") for i in range(3)]
    try:
        dpmod.DataParallel._replay_overlapped(obj, jobs, streams)
    finally:
        pool.shutdown()
    for i in range(3):
        assert [e[2] for e in log if e[0] == "replay" and e[1] == i] == list(range(nseg))
    assert [e[1:] for e in log if e[0] == "reduce"] == [(0, 10), (10, 20), (20, 30)]
    for lo_hi, last_seg in (((0, 10), 2), ((10, 20), 4), ((20, 30), 8)):
        at = log.index(("reduce",) + lo_hi)
        done = [e for e in log[:at] if e[0] == "replay" and e[2] == last_seg]
        assert len(done) == 3, lo_hi
    if threaded:
        assert calls == [3, 3, 3], calls   # three reduce intervals, one task per device each
    else:
        assert calls == []
