"""Stem BN+ReLU+3x3/2 max-pool pass at batch 400 (y0 [400,112,112,64] bf16 -> [400,56,56,64] +
argmax bytes): median of 5 rounds x 10 reps (us) and the achieved bytes/s.
Usage (GPU box): python tools/stem_pool_bench.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402


def main():
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    y = torch.randn(400, 112, 112, 64, device=dev).to(torch.bfloat16)
    sc = torch.rand(64, device=dev) + 0.5
    sh = torch.randn(64, device=dev) * 0.1
    out = torch.empty(400, 56, 56, 64, device=dev, dtype=torch.bfloat16)
    arg = torch.empty(400, 56, 56, 64, device=dev, dtype=torch.uint8)
    for _ in range(3):
        K.stem_pool(y, sc, sh, out, arg)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        st.record()
        for _ in range(10):
            K.stem_pool(y, sc, sh, out, arg)
        en.record()
        en.synchronize()
        ts.append(st.elapsed_time(en) / 10 * 1e3)
    us = statistics.median(ts)
    nbytes = y.numel() * 2 + out.numel() * 2 + arg.numel()
    print(f"stem_pool: {us:.1f} us, {nbytes / us / 1e6:.2f} TB/s")


if __name__ == "__main__":
    main()
