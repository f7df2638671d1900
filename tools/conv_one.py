"""Run one conv shape/pass a few times (for rocprofv3 --pmc runs).
Usage: python tools/conv_one.py <shape> <pass> [reps] [bm] [bn]   e.g. C16 fwd 3"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402
from tools.conv_bench import SHAPES  # noqa: E402


def main():
    name, ps = sys.argv[1], sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    tile = (int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else None
    ext.load(required=True)
    B = 400
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    _, H, Cin, Cout, k, s = next(sh for sh in SHAPES if sh[0] == name)
    g = K.ConvGeom(B, H, H, Cin, Cout, k, k, s, k // 2)
    x = torch.randn(B, H, H, Cin, device=dev).to(dt)
    w = (torch.randn(Cout, k, k, Cin, device=dev) * 0.05).to(dt)
    y = torch.empty(B, g.Ho, g.Wo, Cout, device=dev, dtype=dt)
    dy = torch.randn_like(y)
    dx = torch.empty_like(x)
    gw = torch.empty(Cout * k * k * Cin, device=dev)
    ws = K.Workspace(dev)
    stats = torch.empty(math.ceil(B * g.Ho * g.Wo / 64) * 3 * Cout, device=dev)
    for _ in range(reps):
        if ps == "fwd":
            K.conv_fwd(x, w.view(Cout, -1), g, y, stats=stats, tile=tile)
        elif ps == "dgrad":
            K.conv_dgrad(dy, w, g, dx, tile=tile)
        else:
            K.conv_wgrad(dy, x, g, gw, ws, tile=tile)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
