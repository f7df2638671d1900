"""Calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE against a known byte count.

Runs the BatchNorm apply kernel (csrc/bn.hip bn_apply_u: reads y and the residual, writes the
output; 16-B loads and stores per lane, the access shape of the step's streaming passes and the
conv operand loads) on tensors of a known size, 5 times. Compare each dispatch's FETCH_SIZE /
WRITE_SIZE (KiB) with the printed exact byte counts: MI355X_MICROARCH.md reports FETCH_SIZE at
half the bytes of wide coalesced reads, so the per-step HBM table needs the same factor.
Usage (under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE): python tools/fetch_calib.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402


def main():
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    N, H, C = 400, 56, 256                      # layer1's widest tensor: 642 MB in bf16
    y = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    res = torch.randn_like(y)
    out = torch.empty_like(y)
    sc = torch.rand(C, device=dev) + 0.5
    sh = torch.randn(C, device=dev) * 0.1
    for _ in range(5):
        K.bn_apply(y, sc, sh, out, res=res)
    torch.cuda.synchronize()
    nb = y.numel() * y.element_size()
    print(f"fetch_calib: bn_apply_u exact bytes per launch: read {2 * nb} ({2 * nb / 1024:.0f} KiB), "
          f"write {nb} ({nb / 1024:.0f} KiB)")


if __name__ == "__main__":
    main()
