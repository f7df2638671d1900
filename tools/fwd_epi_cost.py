"""Cost of the conv-forward extras on the output-heavy 1x1 shapes (batch 400): plain forward vs
+ BatchNorm statistics epilogue vs + BN+ReLU operand prologue vs both (the step's form).
Median microseconds per launch, alternating launches.

    python tools/fwd_epi_cost.py"""
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
    B = 400
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    names = sys.argv[1:] or ["C3", "C7", "C13", "C19", "C1", "C4", "C9", "C15", "C21"]
    tot = [0.0] * 4
    for name, H, Cin, Cout, k, s in SHAPES:
        if name not in names:
            continue
        g = K.ConvGeom(B, H, H, Cin, Cout, k, k, s, k // 2)
        x = torch.randn(B, H, H, Cin, device=dev).to(dt)
        w = (torch.randn(Cout, k, k, Cin, device=dev) * 0.05).to(dt).view(Cout, -1)
        y = torch.empty(B, g.Ho, g.Wo, Cout, device=dev, dtype=dt)
        M = B * g.Ho * g.Wo
        stats = torch.empty(K.stats_tiles(M, Cout) * 3 * Cout, device=dev)
        sc, sh = torch.rand(Cin, device=dev) + 0.5, torch.randn(Cin, device=dev) * 0.1
        fns = [lambda: K.conv_fwd(x, w, g, y),
               lambda: K.conv_fwd(x, w, g, y, stats=stats),
               lambda: K.conv_fwd(x, w, g, y, pro=(sc, sh)),
               lambda: K.conv_fwd(x, w, g, y, stats=stats, pro=(sc, sh))]
        ts = [[] for _ in fns]
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for f in fns:
            f()
        torch.cuda.synchronize()
        for _ in range(7):
            for i, f in enumerate(fns):
                ev[0].record()
                for _ in range(5):
                    f()
                ev[1].record()
                torch.cuda.synchronize()
                ts[i].append(ev[0].elapsed_time(ev[1]) * 1e3 / 5)
        med = [statistics.median(t) for t in ts]
        n = COUNT[name]
        for i in range(4):
            tot[i] += n * med[i]
        print(f"{name:4s} {Cout:5d}<-{Cin:5d} k{k} plain {med[0]:7.1f}  +stats {med[1]:7.1f}  "
              f"+pro {med[2]:7.1f}  +both {med[3]:7.1f} us", flush=True)
    print(f"weighted: plain {tot[0]:.0f}  +stats {tot[1]:.0f}  +pro {tot[2]:.0f}  +both {tot[3]:.0f} us")


if __name__ == "__main__":
    main()
