"""Isolated timing of the one-launch BatchNorm statistics kernels (csrc/bn.hip bn_stats_kernel) on
the ResNet-50 batch-400 shapes: forward (shifted conv partials [T][3][C]) and backward (dgrad
epilogue partials [T][2|3][C]). Prints the median microseconds per launch per shape, the
launches-per-step weighted total, and the slab count S used.

    python tools/bnstats_bench.py [--S-scale F]"""
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402

# (M rows, C channels, BN layers of this shape per step) for batch 400
B = 400
FWD = [(B * 112 * 112, 64, 1), (B * 56 * 56, 64, 6), (B * 56 * 56, 256, 4), (B * 56 * 56, 128, 1),
       (B * 28 * 28, 128, 7), (B * 28 * 28, 512, 5), (B * 28 * 28, 256, 1), (B * 14 * 14, 256, 11),
       (B * 14 * 14, 1024, 7), (B * 14 * 14, 512, 1), (B * 7 * 7, 512, 5), (B * 7 * 7, 2048, 4)]


def timeit(fn, inner=20, outer=7):
    """Median over ``outer`` rounds of ``inner`` back-to-back launches (GPU time per launch)."""
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(outer):
        ev[0].record()
        for _ in range(inner):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e3 / inner)
    return statistics.median(ts)


def main():
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    ws = K.Workspace(dev)
    tot_f = tot_b = 0.0
    for M, C_, n in FWD:
        bm = 128
        T = math.ceil(M / bm)
        part = torch.randn(T * 3 * C_, device=dev)
        gamma, beta = torch.rand(C_, device=dev) + 0.5, torch.randn(C_, device=dev)
        st = torch.zeros(4, C_, device=dev)
        rm, rv = torch.zeros(C_, device=dev), torch.ones(C_, device=dev)
        nbt = torch.zeros(1, dtype=torch.long, device=dev)
        bn = K.BnStats(ws, gamma, beta, 1e-5, 0.1, st[0], st[1], st[2], st[3], rm, rv, nbt)
        tf = timeit(lambda: K.bn_finalize_partials(part, T, C_, bm, M, bn))
        # backward: dgrad epilogue partials over the same rows (slabs of 128 rows), nq = 2
        partb = torch.randn(T * 2 * C_, device=dev)
        dg, db = torch.zeros(C_, device=dev), torch.zeros(C_, device=dev)
        S = K._stats_slabs(T, C_)
        slabs = ws.get("bn_slabs", S * 2 * C_, torch.float64)
        cnt = ws.counters(math.ceil(C_ / K._stats_cg(C_)))
        kk = ws.get("bn_k", 6 * C_)
        o = ext.BnBwdOut(float(M), 1.0, 0)
        o.gamma[0], o.mean[0], o.invstd[0] = K.ptr(gamma), K.ptr(st[0]), K.ptr(st[1])
        o.dgamma[0], o.dbeta[0], o.k = K.ptr(dg), K.ptr(db), K.ptr(kk)
        L = ext.lib()

        def bwd():
            K.check(L.pda_bn_bwd_stats(K.ptr(partb), T, 2, C_, S, K.ptr(slabs), K.ptr(cnt),
                                       ext.C.byref(o), K._stats_cg(C_), K.stream(dev)), "bn_bwd_stats")
        tb = timeit(bwd)
        tot_f += n * tf
        tot_b += n * tb
        print(f"M {M:8d} C {C_:5d} T {T:6d} S {S:4d} x{n:2d}  fwd {tf:7.1f} us  bwd {tb:7.1f} us",
              flush=True)
    print(f"weighted per step: fwd {tot_f:.0f} us  bwd {tot_b:.0f} us")
    assert int(ws.counters(16).abs().sum().item()) == 0


if __name__ == "__main__":
    main()
