"""Cost of a cross-stream fork on the issuing stream: N back-to-back launches of one streaming
kernel on the main stream, (a) alone, (b) with an event recorded on the main stream after each
launch, (c) with the second stream waiting on the main stream after each launch (torch
wait_stream = event record + stream wait, what models/native.py _wgrad does per weight gradient),
(d) as (c) plus a small kernel on the second stream per fork. Prints us per main-stream launch.
Usage: python tools/fork_bench.py [n] [MB]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    mb = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    C_ = 256
    rows = mb * (1 << 20) // (2 * C_)
    y = torch.randn(rows, C_, device=dev).to(torch.bfloat16)
    out = torch.empty_like(y)
    sc = torch.rand(C_, device=dev) + 0.5
    sh = torch.randn(C_, device=dev) * 0.1
    small = torch.zeros(1024, device=dev)
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)

    # stream memory operations (HIP, BETA): the main stream writes a counter, the second stream
    # waits for it -- a fork without an event (signal memory from hipExtMallocWithFlags)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    sig = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(sig), ctypes.c_size_t(8), ctypes.c_uint(2))
    if rc != 0:   # (signal memory refused: plain device memory)
        print(f"hipExtMallocWithFlags(signal) rc={rc}; using device memory")
        flag = torch.zeros(2, dtype=torch.int32, device=dev)
        sig = ctypes.c_void_p(flag.data_ptr())
    ms, ss = ctypes.c_void_p(main_s.cuda_stream), ctypes.c_void_p(side.cuda_stream)
    ctr = [0]

    def wv_fork(wait=True):
        ctr[0] += 1
        assert hip.hipStreamWriteValue32(ms, sig, ctypes.c_uint(ctr[0]), ctypes.c_uint(0)) == 0
        if wait:
            assert hip.hipStreamWaitValue32(ss, sig, ctypes.c_uint(ctr[0]), ctypes.c_uint(0),
                                            ctypes.c_uint(0xFFFFFFFF)) == 0

    # the probe kernel (csrc/misc.hip): plain launch, + a torch event record, or launched with a
    # stop event (hipExtLaunchKernel: the dispatch completes it) that the second stream waits on
    L = ext.lib()
    src = torch.randn(mb * (1 << 20) // 8, device=dev)
    dst = torch.empty_like(src)
    evs = []
    for _ in range(n):
        e = ctypes.c_void_p()
        assert hip.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(2)) == 0   # DisableTiming
        evs.append(e)

    def probe(stop=None):
        assert L.pda_fork_probe(dst.data_ptr(), src.data_ptr(), src.numel(), stop, ms) == 0

    def run(mode):
        if mode.startswith("probe"):
            for i in range(n):
                if mode == "probe":
                    probe()
                elif mode == "probe+fork":
                    probe()
                    side.wait_stream(main_s)
                elif mode == "probe+stopev":   # the dispatch's own completion is the fork point
                    probe(evs[i])
                    assert hip.hipStreamWaitEvent(ss, evs[i], ctypes.c_uint(0)) == 0
                elif mode == "probe+stopev-nowait":   # every launch completes an event, no fork
                    probe(evs[i])
                else:   # probe+stopev/5: every launch completes the same event, a fork every 5th
                    probe(evs[0])
                    if i % 5 == 4:
                        assert hip.hipStreamWaitEvent(ss, evs[0], ctypes.c_uint(0)) == 0
            main_s.wait_stream(side)
            return
        for _ in range(n):
            K.bn_apply(y, sc, sh, out, relu=True)
            if mode == "event":
                torch.cuda.Event().record(main_s)
            elif mode in ("fork", "fork+side"):
                side.wait_stream(main_s)
                if mode == "fork+side":
                    with torch.cuda.stream(side):
                        small.add_(1.0)
            elif mode == "write":
                wv_fork(wait=False)
            elif mode in ("wvfork", "wvfork+side"):
                wv_fork()
                if mode == "wvfork+side":
                    with torch.cuda.stream(side):
                        small.add_(1.0)
        main_s.wait_stream(side)

    res = {}
    for rep in range(3):
        for mode in ("plain", "event", "fork", "fork+side", "write", "wvfork", "wvfork+side",
                     "probe", "probe+fork", "probe+stopev", "probe+stopev-nowait", "probe+stopev/5"):
            run(mode)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run(mode)
            b.record()
            torch.cuda.synchronize()
            res.setdefault(mode, []).append(a.elapsed_time(b) * 1e3 / n)
    for mode, v in res.items():
        base = statistics.median(res["probe" if mode.startswith("probe") else "plain"])
        m = statistics.median(v)
        print(f"{mode:10s} {m:8.2f} us per launch  (+{m - base:5.2f})  [{mb} MB bn_apply]")


if __name__ == "__main__":
    main()
