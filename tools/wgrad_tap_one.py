"""Run one 3x3 weight gradient a few times at batch 400 (rocprofv3 --pmc runs): the tap-reuse
kernel or the generic plan. Usage: python tools/wgrad_tap_one.py <C2|C10|C16|C22> <tap|generic> [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402

CASES = {"C2": (56, 64, True), "C10": (28, 128, False), "C16": (14, 256, False), "C22": (7, 512, False)}


def main():
    name, which = sys.argv[1], sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    H, C, pro = CASES[name]
    B = 400
    g = K.ConvGeom(B, H, H, C, C, 3, 3, 1, 1)
    x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
    dy = (torch.randn(B, H, H, C, device=dev) * 0.1).to(torch.bfloat16)
    p = (torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.3) if pro else None
    gw = torch.empty(C * 9 * C, device=dev)
    ws = K.Workspace(dev)
    for _ in range(reps):
        if which == "tap":
            K.conv_wgrad_tap(dy, x, g, gw, ws, pro=p)
        else:
            K._WGRAD_TAP = set()
            K.conv_wgrad(dy, x, g, gw, ws, pro=p)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
