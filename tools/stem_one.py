"""Run the stem conv or the layer1 3x3 conv forward a few times at batch 400 (for rocprofv3 --pmc
runs): python tools/stem_one.py {stem|stem_generic|tap|tap_generic} [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402


def main():
    which = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    B = 400
    if which.startswith("stem"):
        g = K.stem_s2d_geom(B, 224)
        x = (torch.randn(B, 112, 112, 16, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(64, 256, device=dev) * 0.05).to(torch.bfloat16)
        pro = None
    else:
        g = K.ConvGeom(B, 56, 56, 64, 64, 3, 3, 1, 1)
        x = torch.randn(B, 56, 56, 64, device=dev).to(torch.bfloat16)
        w = (torch.randn(64, 576, device=dev) / 24).to(torch.bfloat16)
        pro = (torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.3)
    y = torch.empty(B, g.Ho, g.Wo, 64, device=dev, dtype=torch.bfloat16)
    stats = torch.empty(B * g.Ho * g.Wo // 32 * 3 * 64, device=dev)
    for _ in range(reps):
        if which == "stem":
            K.stem_fwd(x, w, g, y, stats)
        else:
            K.conv_fwd(x, w, g, y, stats=stats, tile=(-128, 64), pro=pro)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
