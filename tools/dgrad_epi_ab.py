"""Cost of the fused BatchNorm-backward dgrad epilogue, shape by shape, on one device: a plain
dgrad (dX stored) vs the same dgrad storing dz = relu-mask(dX [+ g2]) and emitting the BN-backward
partial sums (mode 0: relu(bn(y)); mode 3: the tail form with the forward's ReLU bitmask and a
second gradient source), alternating launches. Prints median microseconds and the COUNT-weighted
totals (tools/conv_bench.py SHAPES / COUNT).

    python tools/dgrad_epi_ab.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402
from tools.conv_bench import COUNT, SHAPES  # noqa: E402


def main():
    ext.load(required=True)
    B = int(os.environ.get("BATCH", "400"))
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    ws = K.Workspace(dev)
    tot = [0.0, 0.0, 0.0]
    for name, H, Cin, Cout, k, s in SHAPES:
        g = K.ConvGeom(B, H, H, Cin, Cout, k, k, s, k // 2)
        dy = torch.randn(B, g.Ho, g.Wo, Cout, device=dev).to(dt)
        w = (torch.randn(Cout, k, k, Cin, device=dev) * 0.05).to(dt)
        y = torch.randn(B, H, H, Cin, device=dev).to(dt)
        g2 = torch.randn_like(y)
        dx = torch.empty_like(y)
        sc, sh = torch.rand(Cin, device=dev) + 0.5, torch.randn(Cin, device=dev) * 0.1
        mask = torch.empty(y.numel() // 8, dtype=torch.uint8, device=dev)
        K.bn_apply(y, sc, sh, torch.empty_like(y), res=g2, mask=mask)
        G = K.dgrad_slabs(g, B)
        epi0, _, _ = K.bn_epilogue(ws, G, y, sc, sh)
        epi3, _, _ = K.bn_epilogue(ws, G, y, sc, sh, g2=g2, mask=mask)
        fns = [lambda: K.conv_dgrad(dy, w, g, dx), lambda: K.conv_dgrad(dy, w, g, dx, epi=epi0),
               lambda: K.conv_dgrad(dy, w, g, dx, epi=epi3)]
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ts = [[], [], []]
        for it in range(10):
            for i, fn in enumerate(fns):
                ev[0].record()
                fn()
                ev[1].record()
                torch.cuda.synchronize()
                if it >= 2:
                    ts[i].append(ev[0].elapsed_time(ev[1]) * 1e3)
        m = [statistics.median(t) for t in ts]
        for i in range(3):
            tot[i] += COUNT[name] * m[i]
        print(f"{name:4s} {Cin:5d}<-{Cout:5d} k{k} s{s}  plain {m[0]:7.1f}  epi0 {m[1]:7.1f} "
              f"({100 * (m[1] / m[0] - 1):+5.1f}%)  epi3 {m[2]:7.1f} ({100 * (m[2] / m[0] - 1):+5.1f}%)",
              flush=True)
    print(f"weighted: plain {tot[0]:.0f} us  epi0 {tot[1]:.0f} us  epi3 {tot[2]:.0f} us")


if __name__ == "__main__":
    main()
