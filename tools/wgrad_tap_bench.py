"""Isolated weight gradient of the ResNet-50 3x3 stride-1 convs at batch 400: the generic
implicit-GEMM plan of the step (tile, split-K, reduce) vs the tap-reuse kernel (csrc/wgrad_tap.hip)
at several block counts. Median of 5 rounds x 5 reps, us (kernel + split-K reduce).
Usage (GPU box): python tools/wgrad_tap_bench.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402

CASES = [("C2", 56, 64, True), ("C10", 28, 128, False), ("C16", 14, 256, False), ("C22", 7, 512, False)]


def timeit(fn, reps=5, rounds=5):
    fn()
    out = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1000.0 / reps)
    return statistics.median(out)


def main():
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    B = 400
    dt = torch.bfloat16
    for name, H, C, pro in CASES:
        g = K.ConvGeom(B, H, H, C, C, 3, 3, 1, 1)
        x = torch.randn(B, H, H, C, device=dev).to(dt)
        dy = (torch.randn(B, H, H, C, device=dev) * 0.1).to(dt)
        p = (torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.3) if pro else None
        gw = torch.empty(C * 9 * C, device=dev)
        ws = K.Workspace(dev)
        old = K._WGRAD_TAP
        K._WGRAD_TAP = set()
        res = {"generic": timeit(lambda: K.conv_wgrad(dy, x, g, gw, ws, pro=p))}
        K._WGRAD_TAP = old
        for blocks in (256, 512):
            old_b = K._WGRAD_TAP_BLOCKS
            def tap(blocks=blocks):
                kb, splits = K.wgrad_tap_plan(g, B, blocks)
                slab = ws.get("wgrad_slab", splits * C * 9 * C)
                L = ext.lib()
                st = K.stream(dev)
                K.check(L.pda_wgrad_tap(K.ptr(dy), K.ptr(x), K.ptr(slab), K.ptr(p[0] if p else None),
                                        K.ptr(p[1] if p else None), B, H, H, C, C, kb, splits, 1, st), "tap")
                K.check(L.pda_wgrad_reduce(K.ptr(slab), K.ptr(gw), splits, C, 9 * C, C.bit_length() - 1,
                                           C, 9 * C, 1.0, 0, None, None, None, st), "red")
            res[f"tap {blocks}"] = timeit(tap)
        print(name, "  ".join(f"{k} {v:7.1f}" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
