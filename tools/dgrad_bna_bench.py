"""DGRAD_BNA vs (apply pass + plain dgrad) on the bottleneck conv1 shapes at batch 400, alone:
microseconds per launch (median of reps), for the plain dgrad, the apply pass, and the folded
dgrad (with dY write-out). Usage: python tools/dgrad_bna_bench.py [reps]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402


def t(fn, reps):
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    ws = K.Workspace(dev)
    for (H, Cin, Cout) in [(56, 256, 64), (56, 64, 64), (28, 512, 128), (14, 1024, 256), (7, 2048, 512)]:
        Nb = 400
        g = K.ConvGeom(Nb, H, H, Cin, Cout, 1, 1, 1, 0)
        dz = torch.randn(Nb, H, H, Cout, device=dev).to(dt)
        y = torch.randn(Nb, H, H, Cout, device=dev).to(dt)
        k = torch.randn(3 * Cout, device=dev)
        w = (torch.randn(Cout, 1, 1, Cin, device=dev) / 16).to(dt)
        dy = torch.empty_like(dz)
        dx = torch.empty(Nb, H, H, Cin, device=dev, dtype=dt)
        tile = K.dgrad_bna_tile(g, Nb)
        a = t(lambda: K.conv_dgrad(dz, w, g, dx, tile=tile), reps)
        b = t(lambda: K.conv_dgrad(dz, w, g, dx, tile=tile, bna=(y, k, dy)), reps)
        c = t(lambda: K.conv_dgrad(dz, w, g, dx, tile=tile, bna=(y, k, None)), reps)
        print(f"H={H} Cin={Cin} Cout={Cout} tile={tile}: plain {a:7.1f} us  bna+write {b:7.1f} us  "
              f"bna {c:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
