"""Per-shape timing of the implicit-GEMM conv kernels on the 23 ResNet-50 conv shapes (+stem, fc)
at batch 400, for every tile configuration. Prints TF/s and the best tile per (shape, pass).
Usage: python tools/conv_bench.py [batch] [reps]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402

SHAPES = [  # name, H, Cin, Cout, k, stride
    ("C1", 56, 64, 64, 1, 1), ("C2", 56, 64, 64, 3, 1), ("C3", 56, 64, 256, 1, 1),
    ("C4", 56, 256, 64, 1, 1), ("C5", 56, 256, 128, 1, 1), ("C6", 56, 128, 128, 3, 2),
    ("C7", 28, 128, 512, 1, 1), ("C8", 56, 256, 512, 1, 2), ("C9", 28, 512, 128, 1, 1),
    ("C10", 28, 128, 128, 3, 1), ("C11", 28, 512, 256, 1, 1), ("C12", 28, 256, 256, 3, 2),
    ("C13", 14, 256, 1024, 1, 1), ("C14", 28, 512, 1024, 1, 2), ("C15", 14, 1024, 256, 1, 1),
    ("C16", 14, 256, 256, 3, 1), ("C17", 14, 1024, 512, 1, 1), ("C18", 14, 512, 512, 3, 2),
    ("C19", 7, 512, 2048, 1, 1), ("C20", 14, 1024, 2048, 1, 2), ("C21", 7, 2048, 512, 1, 1),
    ("C22", 7, 512, 512, 3, 1),
]
COUNT = {"C1": 1, "C2": 3, "C3": 4, "C4": 2, "C5": 1, "C6": 1, "C7": 4, "C8": 1, "C9": 3, "C10": 3,
         "C11": 1, "C12": 1, "C13": 6, "C14": 1, "C15": 5, "C16": 5, "C17": 1, "C18": 1, "C19": 3,
         "C20": 1, "C21": 2, "C22": 2}
TILES = [(128, 128), (128, 64), (64, 128), (64, 64), (-128, 128), (-128, 64), (-64, 128), (-256, 128),
         (1256, 128), (1128, 256), (1128, 128), (2256, 128), (2256, 64)]
# -bm: 1-stage; the -256 tile is compiled for wgrad only (other passes report n/a);
# 1000 + bm: the LDS-DMA 8-wave tiles; 2000 + bm: their tap-reuse form (3x3 stride-1 fwd / dgrad)


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    ws = K.Workspace(dev)
    total_best = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    total_def = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    print(f"{'shape':5s} {'pass':6s} " + " ".join(f"{a:5d}x{b:<3d}" for a, b in TILES) +
          "  default (tile)  best")
    only = set(sys.argv[3].split(",")) if len(sys.argv) > 3 else None
    for name, H, Cin, Cout, k, s in SHAPES:
        if only and name not in only:
            continue
        g = K.ConvGeom(B, H, H, Cin, Cout, k, k, s, k // 2)
        x = torch.randn(B, H, H, Cin, device=dev).to(dt)
        w = (torch.randn(Cout, k, k, Cin, device=dev) * 0.05).to(dt)
        y = torch.empty(B, g.Ho, g.Wo, Cout, device=dev, dtype=dt)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        gw = torch.empty(Cout * k * k * Cin, device=dev)
        M = B * g.Ho * g.Wo
        flop = 2.0 * M * Cout * Cin * k * k
        stats = torch.empty(math.ceil(M / 64) * 3 * Cout, device=dev)
        for ps in ("fwd", "dgrad", "wgrad"):
            ts = []
            for t in TILES:
                if ps == "fwd":
                    f = lambda: K.conv_fwd(x, w.view(Cout, -1), g, y, stats=stats, tile=t)
                elif ps == "dgrad":
                    f = lambda: K.conv_dgrad(dy, w, g, dx, tile=t)
                else:
                    f = lambda: K.conv_wgrad(dy, x, g, gw, ws, tile=t)
                if (t == (-256, 128) and ps != "wgrad") or (t[0] > 2000 and ps == "wgrad"):
                    ts.append(float("inf"))
                    continue
                try:
                    ts.append(timeit(f, reps))
                except RuntimeError:   # geometry the tile does not take (HALO: 3x3 stride 1 only)
                    ts.append(float("inf"))
            if ps == "fwd":
                dflt = K.fwd_tile(g, B, dt)
            elif ps == "dgrad":
                dflt = K.dgrad_tile(g, B)
            else:
                bm, bn, _, _ = K.wgrad_plan(g, B, dma=True)
                dflt = (bm, bn)
            if tuple(dflt) in TILES:
                td = ts[TILES.index(tuple(dflt))]
            else:   # a default tile outside the sweep list (e.g. the 256x256 weight-gradient tile)
                t = tuple(dflt)
                if ps == "fwd":
                    f = lambda: K.conv_fwd(x, w.view(Cout, -1), g, y, stats=stats, tile=t)
                elif ps == "dgrad":
                    f = lambda: K.conv_dgrad(dy, w, g, dx, tile=t)
                else:
                    f = lambda: K.conv_wgrad(dy, x, g, gw, ws, tile=t)
                td = timeit(f, reps)
            tb = min(min(ts), td)
            n = COUNT[name]
            total_best[ps] += tb * n
            total_def[ps] += td * n
            print(f"{name:5s} {ps:6s} " + " ".join(f"{v:9.1f}" for v in ts) +
                  f"  {td:7.1f} {str(tuple(dflt)):>12s}  "
                  f"{(TILES[ts.index(tb)] if tb in ts else tuple(dflt))} {flop / tb / 1e6:6.0f}TF")
    print("per-step totals (us, x layer count): default", {k: round(v) for k, v in total_def.items()},
          " best", {k: round(v) for k, v in total_best.items()})


if __name__ == "__main__":
    main()
