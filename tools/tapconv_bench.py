"""Layer1 conv2 forward (3x3/1/1, 64 -> 64, 56x56, batch 400) with the BN+ReLU prologue and the
BN-statistics epilogue as in the step: csrc/tapconv.hip (persistent-block sweep) vs the generic
register tile. Median of 5 rounds x 5 reps (us). Usage (GPU box): python tools/tapconv_bench.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402


def timeit(fn):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        st.record()
        for _ in range(5):
            fn()
        en.record()
        en.synchronize()
        ts.append(st.elapsed_time(en) / 5 * 1e3)
    return statistics.median(ts)


def main():
    ext.load(required=True)
    B, H, C = 400, 56, 64
    dev = torch.device("cuda", 0)
    g = K.ConvGeom(B, H, H, C, C, 3, 3, 1, 1)
    x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(C, 576, device=dev) / 24).to(torch.bfloat16)
    sc = torch.rand(C, device=dev) + 0.5
    sh = torch.randn(C, device=dev) * 0.3
    y = torch.empty(B, H, H, C, device=dev, dtype=torch.bfloat16)
    stats = torch.empty(B * H * H // 64 * 3 * C, device=dev)
    print(f"layer1 conv2 fwd M={B * H * H} N=64 K=576, BN prologue + statistics")
    for cap in (128, 256, 512, 700, 1400, 2800):
        def run(c=cap):
            K.check(ext.lib().pda_tapconv_fwd(K.ptr(x), K.ptr(w), K.ptr(y), K.ptr(stats), K.ptr(sc),
                                              K.ptr(sh), B, H, H, 1, c, K.stream(dev)), "tapconv")
        print(f"  csrc/tapconv.hip grid cap {cap}: {timeit(run):8.1f} us")
    for t in [(-128, 64), (128, 64), (-128, 128)]:
        print(f"  generic tile {t}: "
              f"{timeit(lambda t=t: K.conv_fwd(x, w, g, y, stats=stats, tile=t, pro=(sc, sh))):8.1f} us")


if __name__ == "__main__":
    main()
