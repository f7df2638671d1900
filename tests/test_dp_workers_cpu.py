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
