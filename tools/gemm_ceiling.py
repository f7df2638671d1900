"""Library-GEMM ceiling for the 1x1 ResNet-50 conv shapes: torch.mm (hipBLASLt, bf16) on the
equivalent [M, K] x [K, N] problem next to our conv kernels' default tile for the same pass.
A 1x1 stride-1 conv IS that GEMM, so hipBLASLt's time is the bar our implicit-GEMM kernels are
measured against. Usage: python tools/gemm_ceiling.py [batch] [reps]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402
from tools.conv_bench import SHAPES, timeit  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    from pytorch_distributed_amd.ops import ext
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    a = torch.randn(8192, 8192, device=dev).to(dt)
    t = timeit(lambda: torch.mm(a, a), reps)
    print(f"hipBLASLt 8192^3 bf16: {t:.1f} us, {2 * 8192 ** 3 / t / 1e6:.0f} TF/s")
    del a
    print(f"{'shape':6s} {'pass':6s} {'M':>7s} {'N':>5s} {'K':>5s} {'hipBLASLt us':>13s} {'TF':>5s} "
          f"{'ours us':>8s} {'TF':>5s} {'tile':>12s}")
    for name, H, Cin, Cout, k, s in SHAPES:
        if k != 1 or s != 1:
            continue
        g = K.ConvGeom(B, H, H, Cin, Cout, 1, 1, 1, 0)
        M = B * H * H
        x = torch.randn(B, H, H, Cin, device=dev).to(dt)
        w = (torch.randn(Cout, Cin, device=dev) * 0.05).to(dt)
        y = torch.empty(B, H, H, Cout, device=dev, dtype=dt)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        stats = torch.empty(math.ceil(M / 64) * 3 * Cout, device=dev)
        x2, dy2, wt = x.view(M, Cin), dy.view(M, Cout), w.t().contiguous()
        for ps in ("fwd", "dgrad"):
            if ps == "fwd":
                tile = K.fwd_tile(g, B, dt)
                lib = lambda: torch.mm(x2, wt)              # noqa: E731  [M,Cin] x [Cin,Cout]
                ours = lambda: K.conv_fwd(x, w, g, y, stats=stats, tile=tile)  # noqa: E731
                Mg, Ng, Kg = M, Cout, Cin
            else:
                tile = K.dgrad_tile(g, B)
                lib = lambda: torch.mm(dy2, w)              # noqa: E731  [M,Cout] x [Cout,Cin]
                ours = lambda: K.conv_dgrad(dy, w.view(Cout, 1, 1, Cin), g, dx, tile=tile)  # noqa: E731
                Mg, Ng, Kg = M, Cin, Cout
            fl = 2.0 * Mg * Ng * Kg
            tl, to = timeit(lib, reps), timeit(ours, reps)
            print(f"{name:6s} {ps:6s} {Mg:7d} {Ng:5d} {Kg:5d} {tl:13.1f} {fl / tl / 1e6:5.0f} "
                  f"{to:8.1f} {fl / to / 1e6:5.0f} {str(tile):>12s}", flush=True)


if __name__ == "__main__":
    main()
