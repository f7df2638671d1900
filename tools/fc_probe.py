"""The ResNet-50 head's fc launches at batch 400 (M = 400 rows, K = 2048, N = 1000 classes: a GEMM
too small to fill 256 CUs with the default tile) on every built tile: forward (f32 logits + bias)
and data gradient, us per launch (median of 50).

    python tools/fc_probe.py
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) * 1e3 for a, b in ev)


def main() -> None:
    from pytorch_distributed_amd.ops import ext
    from pytorch_distributed_amd.ops import native_ops as K
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    B, F_, NC, NR = 400, 2048, 1000, 1024   # NR: fc rows padded as the model pads them
    feat = torch.randn(B, F_, device=dev).to(torch.bfloat16)
    w = (torch.randn(NR, F_, device=dev) * 0.02).to(torch.bfloat16)
    bias = torch.randn(NC, device=dev)
    logits = torch.empty(B, NC, device=dev)
    g = K.ConvGeom(B, 1, 1, F_, NC, 1, 1, 1, 0)
    print("default fwd tile", K.fwd_tile(g, B, torch.bfloat16))
    ref = None
    for tile in (None, (64, 128), (64, 64), (128, 64), (-64, 128), (-128, 64)):
        try:
            fn = lambda: K.conv_fwd(feat, w, g, logits, bias=bias, tile=tile)
            fn()
            torch.cuda.synchronize()
        except Exception as e:   # noqa: BLE001 (tile not built for this pass)
            print(f"fwd tile {tile}: {e}")
            continue
        if ref is None:
            ref = logits.clone()
        err = (logits - ref).abs().max().item()
        print(f"fwd tile {str(tile):12s} {timeit(fn):7.1f} us  max|diff| {err:.2e}")
    dlog = torch.randn(B, NR, device=dev).to(torch.bfloat16)
    dx = torch.empty(B, 1, 1, F_, device=dev, dtype=torch.bfloat16)
    gd = K.ConvGeom(B, 1, 1, F_, NR, 1, 1, 1, 0)
    w4 = w.view(NR, 1, 1, F_)
    for tile in (None, (64, 128), (64, 64), (128, 64), (-64, 128)):
        try:
            fn = lambda: K.conv_dgrad(dlog.view(B, 1, 1, NR), w4, gd, dx, tile=tile)
            fn()
            torch.cuda.synchronize()
        except Exception as e:   # noqa: BLE001
            print(f"dgrad tile {tile}: {e}")
            continue
        print(f"dgrad tile {str(tile):12s} {timeit(fn):7.1f} us")
    print("fc_probe: ok")


if __name__ == "__main__":
    main()
