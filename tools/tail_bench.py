"""Isolated cost of a block tail + the next block's conv1 forward at batch 400: the apply pass
(bn_apply, residual + ReLU + bitmask) followed by the plain conv, against the fused FWD_TAIL conv
(csrc/conv_gemm.hip) on 128x64 and 128x128 tiles. Median of 5 rounds x 5 reps, us.
Usage (GPU box): python tools/tail_bench.py"""
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402

# (name, H, Cin = tail channels, Cout = conv1 channels)
CASES = [("layer1", 56, 256, 64), ("layer2", 28, 512, 128), ("layer3", 14, 1024, 256),
         ("layer4", 7, 2048, 512)]


def timeit(fn, reps=5, rounds=5):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(rounds)]
    fn()
    out = []
    for a, b in ev:
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1000.0 / reps)
    return statistics.median(out)


def main():
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    B = 400
    dt = torch.bfloat16
    for name, H, Cin, Cout in CASES:
        g = K.ConvGeom(B, H, H, Cin, Cout, 1, 1, 1, 0)
        y3 = torch.randn(B, H, H, Cin, device=dev).to(dt)
        r = torch.randn_like(y3)
        a = torch.empty_like(y3)
        m = torch.empty(y3.numel() // 8, dtype=torch.uint8, device=dev)
        sc, sh = torch.rand(Cin, device=dev) + 0.5, torch.randn(Cin, device=dev) * 0.3
        w = (torch.randn(Cout, Cin, device=dev) / math.sqrt(Cin)).to(dt)
        y = torch.empty(B, H, H, Cout, device=dev, dtype=dt)
        T = math.ceil(B * H * H / 64)
        st = torch.empty(T * 3 * Cout, device=dev)
        tile = K.fwd_tile(g, B, dt)

        def unfused():
            K.bn_apply(y3, sc, sh, a, res=r, mask=m)
            K.conv_fwd(a, w, g, y, stats=st, tile=tile)
        res = {"apply+conv": timeit(unfused)}
        for bn in (64, 128):
            if bn == 128 and Cout < 128:
                continue
            def fused(bn=bn):
                K.check(ext.lib().pda_conv_fwd_tail(
                    ext.C.byref(g.desc(B)), K.ptr(y3), K.ptr(w), Cin, K.ptr(y), K.ptr(st), K.ptr(sc),
                    K.ptr(sh), K.ptr(r), None, None, K.ptr(a), K.ptr(m), 1, 1, -128, bn,
                    K.stream(dev)), "tail")
            res[f"fused 128x{bn}"] = timeit(fused)
        res["apply alone"] = timeit(lambda: K.bn_apply(y3, sc, sh, a, res=r, mask=m))
        res[f"conv alone {tile}"] = timeit(lambda: K.conv_fwd(a, w, g, y, stats=st, tile=tile))
        print(name, "  ".join(f"{k} {v:7.1f}" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
