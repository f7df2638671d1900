"""Python side of the native RCCL communicator (``csrc/comm/rccl_comm.cpp``).

Multi-process: the ``ncclUniqueId`` of rank 0 is exchanged through the default
``torch.distributed`` TCPStore, then every rank runs ``ncclCommInitRank``.
Collectives run on a dedicated HIP stream (default priority, see ``__init__``): ``all_reduce_async``
records an event on the compute stream, makes the comm stream wait on it,
enqueues ``ncclAllReduce`` and returns a completion event; ``wait`` makes the
*current* stream wait on that event (the host never blocks). This is how DDP
gradient buckets overlap the rest of backward.

Single-process multi-GPU (DataParallel): :class:`RcclGroup` wraps
``ncclCommInitAll`` and issues one grouped collective across all devices.
"""
from __future__ import annotations

import ctypes as C
import itertools
import os
from pathlib import Path
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from .comm import Communicator

__all__ = ["CommAbortedError", "RcclBucketReducer", "RcclCommunicator", "RcclGroup", "load"]

LIBPATH = Path(__file__).resolve().parent.parent / "_lib" / "libpda_comm.so"
_LIB: Optional[C.CDLL] = None
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int64: 3, torch.float64: 4,
       torch.int32: 5, torch.uint8: 6}
ERR_ABORTED = 1001   # csrc/comm/comm.h kErrAborted
_OPS = {"sum": 0, "avg": 1, "max": 2, "min": 3}
_gen = itertools.count()


def load() -> C.CDLL:
    global _LIB
    if _LIB is None:
        if not LIBPATH.exists() and os.environ.get("PDA_NO_BUILD") != "1":
            from .. import _build
            _build.build_comm()
        lib = C.CDLL(str(LIBPATH))
        V, I, Z = C.c_void_p, C.c_int, C.c_size_t
        sigs = {
            "pda_comm_unique_id": [C.c_char_p],
            "pda_comm_init_rank": [C.c_char_p, I, I, I, C.POINTER(V)],
            "pda_comm_init_all": [C.POINTER(I), I, C.POINTER(V)],
            "pda_comm_destroy": [V, I],
            "pda_comm_abort": [V, I],
            "pda_comm_is_aborted": [V],
            "pda_comm_check": [V],
            "pda_comm_count": [V, C.POINTER(I)],
            "pda_allreduce": [V, V, V, Z, I, I, V],
            "pda_broadcast": [V, V, V, Z, I, I, V],
            "pda_reduce": [V, V, V, Z, I, I, I, V],
            "pda_allgather": [V, V, V, Z, I, V],
            "pda_reduce_scatter": [V, V, V, Z, I, I, V],
            "pda_group_allreduce": [V, C.POINTER(V), Z, I, I, C.POINTER(V)],
            "pda_group_broadcast": [V, C.POINTER(V), Z, I, I, C.POINTER(V)],
            "pda_group_reduce": [V, C.POINTER(V), Z, I, I, I, C.POINTER(V)],
            "pda_reducer_create": [V, V, I, I, C.POINTER(C.c_longlong), I, V, C.POINTER(V)],
            "pda_reducer_ready": [V, C.c_longlong, V],
            "pda_reducer_finish": [V, V, V],
            "pda_reducer_reset": [V],
            "pda_reducer_destroy": [V],
            "pda_reducer_num_buckets": [V],
            "pda_reducer_set_timing": [V, I],
            "pda_reducer_timing": [V, C.POINTER(C.c_float)],
        }
        for n, a in sigs.items():
            f = getattr(lib, n)
            f.argtypes = a
            f.restype = I
        lib.pda_reducer_launched.argtypes = [V]
        lib.pda_reducer_launched.restype = C.c_longlong
        lib.pda_comm_error_string.argtypes = [I]
        lib.pda_comm_error_string.restype = C.c_char_p
        _LIB = lib
    return _LIB


class CommAbortedError(RuntimeError):
    """The communicator was aborted (watchdog saw an asynchronous error, or it was closed)."""


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().pda_comm_error_string(rc).decode()
        cls = CommAbortedError if rc == ERR_ABORTED else RuntimeError
        raise cls(f"RCCL {what} failed: {msg} ({rc})")


class RcclCommunicator(Communicator):
    supports_avg = True

    def __init__(self, device: torch.device, group=None, store=None) -> None:
        if not dist.is_initialized():
            raise RuntimeError("RcclCommunicator needs an initialised torch.distributed (for the store)")
        lib = load()
        self.device = torch.device(device)
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        store = store if store is not None else dist.distributed_c10d._get_default_store()
        key = f"pda_rccl_uid_{next(_gen)}"
        if self.rank == 0:
            buf = C.create_string_buffer(128)
            _check(lib.pda_comm_unique_id(buf), "get_unique_id")
            store.set(key, bytes(buf.raw))
            uid = bytes(buf.raw)
        else:
            uid = store.get(key)
        self._h = C.c_void_p()
        self._init_rank(lib, uid)
        # default priority: a high-priority comm stream (priority -1) made every DDP step 13-15 ms
        # slower at the image's GPU_MAX_HW_QUEUES=4 (28.8 -> 43.3 ms/step, ResNet-50 bs 400; fine
        # at 3, 6 or 8 queues, 32.0 at 5): the HIP runtime's queue mapping for a second priority
        # level, not the collectives, cost it (tools/ddp_sync_diag.py, profiles/ddp_overhead_r3.md).
        self.stream = torch.cuda.Stream(self.device, priority=0)
        self._watchdog_error = None
        self._watchdog = None
        self._watchdog_stop = None

    def _init_rank(self, lib, uid: bytes) -> None:
        """``ncclCommInitRank`` blocks until every rank has joined; run it with a deadline
        (``PDA_RCCL_INIT_TIMEOUT_S``, default 600 s) so a missing or mismatched rank becomes a
        clear error instead of a silent hang (ctypes releases the GIL during the call)."""
        import threading
        timeout = float(os.environ.get("PDA_RCCL_INIT_TIMEOUT_S", "600"))
        res = {}

        def run():
            res["rc"] = lib.pda_comm_init_rank(uid, self.world_size, self.rank, self.device.index,
                                               C.byref(self._h))
        t = threading.Thread(target=run, name="rccl-init", daemon=True)
        t.start()
        t.join(timeout)
        if t.is_alive():
            raise TimeoutError(f"ncclCommInitRank did not complete within {timeout:.0f} s on rank "
                               f"{self.rank}/{self.world_size} (a rank missing or stuck?)")
        _check(res["rc"], "init_rank")

    def _live(self) -> C.c_void_p:
        """The native handle, or raise if the communicator was closed / aborted by the watchdog."""
        if not self._h or self._watchdog_error is not None:
            self.check()
        return self._h

    @property
    def rccl_count(self) -> int:
        """Number of ranks RCCL itself reports for this communicator (``ncclCommCount``)."""
        n = C.c_int(0)
        _check(load().pda_comm_count(self._live(), C.byref(n)), "comm_count")
        return int(n.value)

    # async on the comm stream ----------------------------------------------------------
    def all_reduce_async(self, t: torch.Tensor, op: str = "sum"):
        cur = torch.cuda.current_stream(self.device)
        ready = torch.cuda.Event()
        ready.record(cur)
        self.stream.wait_event(ready)
        _check(load().pda_allreduce(self._live(), t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
                                    _OPS[op], self.stream.cuda_stream), "allreduce")
        done = torch.cuda.Event()
        done.record(self.stream)
        t.record_stream(self.stream)
        return done

    def broadcast_async(self, t: torch.Tensor, src: int = 0):
        """Broadcast on the comm stream, ordered after the current stream's work; returns the
        completion event (join with :meth:`wait` where ``t`` is next read or written)."""
        cur = torch.cuda.current_stream(self.device)
        ready = torch.cuda.Event()
        ready.record(cur)
        self.stream.wait_event(ready)
        _check(load().pda_broadcast(self._live(), t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
                                    src, self.stream.cuda_stream), "broadcast")
        done = torch.cuda.Event()
        done.record(self.stream)
        t.record_stream(self.stream)
        return done

    def make_bucket_reducer(self, flat: torch.Tensor, buckets) -> "RcclBucketReducer":
        """Native bucket reducer over contiguous ``(begin, end)`` element ranges of ``flat``."""
        return RcclBucketReducer(self, flat, buckets)

    def wait(self, handle) -> None:
        if self._watchdog_error is not None:
            self.check()
        if handle is not None:
            torch.cuda.current_stream(self.device).wait_event(handle)

    # ordered on the current stream ----------------------------------------------------
    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        st = torch.cuda.current_stream(self.device).cuda_stream
        _check(load().pda_broadcast(self._live(), t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], src,
                                    st), "broadcast")

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> None:
        st = torch.cuda.current_stream(self.device).cuda_stream
        _check(load().pda_allreduce(self._live(), t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
                                    _OPS[op], st), "allreduce")

    def reduce(self, t: torch.Tensor, dst: int = 0, op: str = "sum") -> None:
        st = torch.cuda.current_stream(self.device).cuda_stream
        _check(load().pda_reduce(self._live(), t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], _OPS[op],
                                 dst, st), "reduce")

    def all_gather(self, out: torch.Tensor, t: torch.Tensor) -> None:
        st = torch.cuda.current_stream(self.device).cuda_stream
        _check(load().pda_allgather(self._live(), t.data_ptr(), out.data_ptr(), t.numel(), _DT[t.dtype], st),
               "allgather")

    def barrier(self) -> None:
        t = torch.ones(1, device=self.device)
        self.all_reduce(t)
        torch.cuda.current_stream(self.device).synchronize()

    def check(self) -> None:
        """Raise if the communicator saw an asynchronous error (dead peer, network) or was aborted."""
        err = self._watchdog_error
        if err is not None:
            raise CommAbortedError(f"RCCL communicator aborted by watchdog: {err}")
        if not self._h:
            raise CommAbortedError("RCCL communicator closed")
        _check(load().pda_comm_check(self._h), "async")

    @property
    def aborted(self) -> bool:
        return not self._h or bool(load().pda_comm_is_aborted(self._h))

    def abort(self) -> None:
        """Abort in-flight and future collectives WITHOUT freeing the communicator (that happens in
        :meth:`close` on the owning thread): blocked collectives return, later enqueues -- including
        every bucket launch of a reducer built on it -- fail with :class:`CommAbortedError`."""
        if self._h:
            load().pda_comm_abort(self._h, 2000)

    def start_watchdog(self, interval_s: float = 5.0) -> None:
        """Poll ``ncclCommGetAsyncError`` from a daemon thread; on an error (e.g. a dead peer) abort
        the communicator so collectives blocked on it return instead of hanging, and make the next
        :meth:`check` / :meth:`wait` / bucket launch raise (SURVEY §5.3 failure detection). The
        thread never frees anything (csrc/comm/comm.h lifetime model)."""
        import threading
        stop = threading.Event()
        lib, h = load(), self._h

        def run():
            while not stop.wait(interval_s):
                rc = lib.pda_comm_check(h)
                if rc == ERR_ABORTED:
                    return
                if rc != 0:
                    self._watchdog_error = lib.pda_comm_error_string(rc).decode()
                    lib.pda_comm_abort(h, 2000)
                    return

        self._watchdog_stop = stop
        t = threading.Thread(target=run, name="rccl-watchdog", daemon=True)
        t.start()
        self._watchdog = t

    def stop_watchdog(self) -> None:
        if self._watchdog_stop is not None:
            self._watchdog_stop.set()
        if self._watchdog is not None:
            self._watchdog.join()
        self._watchdog = self._watchdog_stop = None

    def close(self, abort: bool = False) -> None:
        """Stop the watchdog, then drop this handle's reference (reducers built on the
        communicator keep the native struct alive, aborted, until they are closed too)."""
        self.stop_watchdog()
        if self._h:
            h, self._h = self._h, C.c_void_p()
            load().pda_comm_destroy(h, int(abort))


class RcclBucketReducer:
    """Python handle of the C++ gradient-bucket reducer (``csrc/comm/reducer.cpp``).

    ``ready(upto)`` launches, on the communicator's stream, an ncclAvg all-reduce of every bucket
    whose gradients are final (ordered after the current stream by a pre-created HIP event);
    ``finish()`` launches the rest and makes the current stream wait for the last bucket. The
    host never blocks and no Python object is created per bucket."""

    def __init__(self, comm: RcclCommunicator, flat: torch.Tensor, buckets) -> None:
        if not flat.is_contiguous() or flat.dtype not in _DT:
            raise ValueError("flat gradient must be a contiguous tensor of a supported dtype")
        self.comm = comm
        self.flat = flat
        self.buckets = [(int(s), int(e)) for s, e in buckets]
        arr = (C.c_longlong * (2 * len(self.buckets)))(*[v for b in self.buckets for v in b])
        self._h = C.c_void_p()
        _check(load().pda_reducer_create(comm._live(), flat.data_ptr(), _DT[flat.dtype], _OPS["avg"], arr,
                                         len(self.buckets), comm.stream.cuda_stream, C.byref(self._h)),
               "reducer_create")

    def _hh(self) -> C.c_void_p:
        if not self._h:
            raise CommAbortedError("bucket reducer closed")
        return self._h

    def ready(self, upto: int) -> None:
        st = torch.cuda.current_stream(self.comm.device).cuda_stream
        self._rc(load().pda_reducer_ready(self._hh(), int(upto), st), "reducer_ready")

    def finish(self) -> None:
        st = torch.cuda.current_stream(self.comm.device).cuda_stream
        self._rc(load().pda_reducer_finish(self._hh(), st, st), "reducer_finish")

    def _rc(self, rc: int, what: str) -> None:
        if rc == ERR_ABORTED and self.comm._watchdog_error is not None:
            raise CommAbortedError(f"RCCL {what}: communicator aborted by watchdog: "
                                   f"{self.comm._watchdog_error}")
        _check(rc, what)

    def reset(self) -> None:
        load().pda_reducer_reset(self._hh())

    @property
    def launched(self) -> int:
        """Total bucket all-reduces launched since construction."""
        return int(load().pda_reducer_launched(self._h))

    def set_timing(self, on: bool) -> None:
        """Record per-bucket / exposed-communication timing events from the next step on (the
        events cost a few us per bucket: diagnostics only, never in a timed run)."""
        _check(load().pda_reducer_set_timing(self._h, int(bool(on))), "reducer_set_timing")

    def timing(self):
        """After a timed step has completed (synchronise first): ``(exposed_ms, [bucket_ms...])``
        -- exposed = backward end -> last bucket all-reduce done on the comm stream."""
        nb = len(self.buckets)
        out = (C.c_float * (nb + 1))()
        _check(load().pda_reducer_timing(self._h, out), "reducer_timing")
        return float(out[0]), [float(v) for v in out[1:]]

    def close(self) -> None:
        if self._h:
            h, self._h = self._h, C.c_void_p()
            load().pda_reducer_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RcclGroup:
    """In-process communicator over several local GPUs (``ncclCommInitAll``)."""

    def __init__(self, devices: Sequence[int]) -> None:
        lib = load()
        self.devices = list(devices)
        n = len(self.devices)
        arr = (C.c_int * n)(*self.devices)
        self._h = C.c_void_p()
        _check(lib.pda_comm_init_all(arr, n, C.byref(self._h)), "init_all")

    def _streams(self, streams=None):
        n = len(self.devices)
        if streams is None:
            streams = [torch.cuda.current_stream(d) for d in self.devices]
        if len(streams) != n:
            raise ValueError(f"{len(streams)} streams for a group of {n} devices")
        return (C.c_void_p * n)(*[s.cuda_stream for s in streams])

    def _bufs(self, ts: List[torch.Tensor]):
        if len(ts) != len(self.devices) or len({t.numel() for t in ts}) != 1:
            raise ValueError("one tensor of equal size per device of the group")
        return (C.c_void_p * len(ts))(*[t.data_ptr() for t in ts])

    def all_reduce(self, ts: List[torch.Tensor], op: str = "sum", streams=None) -> None:
        """Grouped all-reduce, one tensor per device, enqueued on ``streams`` (default: each
        device's current stream)."""
        _check(load().pda_group_allreduce(self._h, self._bufs(ts), ts[0].numel(), _DT[ts[0].dtype],
                                          _OPS[op], self._streams(streams)), "group_allreduce")

    def broadcast(self, ts: List[torch.Tensor], root: int = 0) -> None:
        _check(load().pda_group_broadcast(self._h, self._bufs(ts), ts[0].numel(), _DT[ts[0].dtype],
                                          root, self._streams()), "group_broadcast")

    def reduce(self, ts: List[torch.Tensor], root: int = 0, op: str = "sum") -> None:
        _check(load().pda_group_reduce(self._h, self._bufs(ts), ts[0].numel(), _DT[ts[0].dtype],
                                       _OPS[op], root, self._streams()), "group_reduce")

    def close(self) -> None:
        if self._h:
            h, self._h = self._h, C.c_void_p()
            load().pda_comm_destroy(h, 0)
