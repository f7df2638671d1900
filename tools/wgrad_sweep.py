"""Split-K sweep for the weight-gradient kernels: for every ResNet-50 conv shape at batch 400,
time conv_wgrad (kernel + slab reduction) for several tiles x target block counts.
Usage: python tools/wgrad_sweep.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402
from tools.conv_bench import COUNT, SHAPES, timeit  # noqa: E402

TILES = [tuple(int(v) for v in t.split(":")) for t in os.environ.get(
    "WS_TILES", "64:64,128:64,64:128,-128:128,128:128,-256:128").split(",")]
TARGETS = [int(v) for v in os.environ.get("WS_TARGETS", "512,1024,2048,4096").split(",")]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    ext.load(required=True)
    B = 400
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    ws = K.Workspace(dev)
    tot_def = tot_best = 0.0
    print("shape  " + " ".join(f"{a:4d}x{b:<3d}/{t:<4d}" for a, b in TILES for t in TARGETS))
    for name, H, Cin, Cout, k, s in SHAPES:
        g = K.ConvGeom(B, H, H, Cin, Cout, k, k, s, k // 2)
        x = torch.randn(B, H, H, Cin, device=dev).to(dt)
        dy = torch.randn(B, g.Ho, g.Wo, Cout, device=dev).to(dt)
        gw = torch.empty(Cout * k * k * Cin, device=dev)
        res = {}
        for t in TILES:
            for tb in TARGETS:
                res[(t, tb)] = timeit(lambda: K.conv_wgrad(dy, x, g, gw, ws, tile=t, target_blocks=tb), reps)
        bm, bn, _, _ = K.wgrad_plan(g, B)
        d = timeit(lambda: K.conv_wgrad(dy, x, g, gw, ws), reps)
        best = min(res, key=res.get)
        tot_def += d * COUNT[name]
        tot_best += res[best] * COUNT[name]
        print(f"{name:5s} " + " ".join(f"{res[(t, tb)]:12.1f}" for t in TILES for tb in TARGETS)
              + f"   default {d:.1f} ({bm},{bn})  best {res[best]:.1f} {best}", flush=True)
        del x, dy, gw
    print(f"per-step wgrad totals (us): default {tot_def:.0f} best {tot_best:.0f}")


if __name__ == "__main__":
    main()
