"""How much of a forward conv is its epilogue: the expansion / reduction 1x1 shapes and a 3x3 at
batch 400, timed with and without the BatchNorm-statistics epilogue (stats=None) and with and
without the BN+ReLU operand prologue, on the default tile. Usage: python tools/fwd_epi_probe.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) * 1e3)
    return statistics.median(out)


def main():
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    for (H, Cin, Cout, k) in [(56, 64, 256, 1), (28, 128, 512, 1), (14, 256, 1024, 1), (7, 512, 2048, 1),
                              (56, 256, 64, 1), (56, 64, 64, 3), (28, 512, 128, 1)]:
        B = 400
        g = K.ConvGeom(B, H, H, Cin, Cout, k, k, 1, k // 2)
        x = torch.randn(B, H, H, Cin, device=dev).to(dt)
        w = (torch.randn(Cout, k * k * Cin, device=dev) * 0.05).to(dt)
        y = torch.empty(B, H, H, Cout, device=dev, dtype=dt)
        M = B * H * H
        st = torch.empty((M // 64 + 1) * 3 * Cout, device=dev)
        pro = (torch.rand(Cin, device=dev) + 0.5, torch.randn(Cin, device=dev) * 0.1)
        tile = K.fwd_tile(g, B, dt, True, k * k * Cin)
        r = {}
        r["stats+pro"] = t(lambda: K.conv_fwd(x, w, g, y, stats=st, pro=pro, tile=tile))
        r["stats"] = t(lambda: K.conv_fwd(x, w, g, y, stats=st, tile=tile))
        r["pro"] = t(lambda: K.conv_fwd(x, w, g, y, pro=pro, tile=tile))
        r["plain"] = t(lambda: K.conv_fwd(x, w, g, y, tile=tile))
        mb = (M * Cin + M * Cout) * 2 / 1e6
        print(f"H={H} {Cin}->{Cout} k={k} tile={tile} MB={mb:.0f}: " +
              "  ".join(f"{a} {v:7.1f} us ({mb / v:.2f} TB/s)" for a, v in r.items()), flush=True)


if __name__ == "__main__":
    main()
