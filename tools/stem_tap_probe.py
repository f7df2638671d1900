"""Three launches each of the stem weight gradient's tap-reuse kernel (512 blocks) and of the
generic WGRAD_BNA tile, at batch 400 -- a short program for a rocprofv3 --pmc pass.
Usage (GPU box): rocprofv3 --kernel-trace --pmc ... -- python3 tools/stem_tap_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402


def main():
    ext.load(required=True)
    B, dev = 400, torch.device("cuda", 0)
    g = K.stem_s2d_geom(B, 224)
    x = (torch.randn(B, 112, 112, 16, device=dev) * 0.5).to(torch.bfloat16)
    dz = (torch.randn(B, 112, 112, 64, device=dev) * 0.01).to(torch.bfloat16)
    y = torch.randn(B, 112, 112, 64, device=dev).to(torch.bfloat16)
    k = torch.randn(3 * 64, device=dev) * 0.1
    ws, out = K.Workspace(dev), torch.empty(64 * 256, device=dev)
    for _ in range(3):
        K.conv_wgrad_stem_tap(dz, y, k, x, g, out, ws, blocks=int(os.environ.get("BLOCKS", "512")))
        K.conv_wgrad(dz, x, g, out, ws, bna=(y, k), tile=(-64, 256), target_blocks=1024)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
