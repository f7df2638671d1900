"""Isolated timing of the 3x3 stride-1 convs of layers 1-2 (C2: 56 px 64 -> 64, C10: 28 px
128 -> 128) at batch 400 on the tile choices the step could use:
  fwd  : generic register-staged tile with the BN+ReLU operand prologue (the step's layer-1 path)
         vs bn_apply (materialise relu(bn(y))) + the tap-reuse HALO tile
         (round 5 also timed a HALO forward applying the prologue to its slab in LDS and a
         one-slab-slot 64-channel HALO: faster alone, slower in the step -- removed,
         profiles/ab_r5.md section 5)
  dgrad: generic tile vs the HALO tile.
Usage: python tools/halo_bench.py [reps]   (prints one line per case, us per launch, median)"""
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402


def timeit(fn, reps):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    fn()
    torch.cuda.synchronize()
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) * 1e3 for a, b in ev)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    B = 400
    for name, H, C_ in (("C2", 56, 64), ("C10", 28, 128)):
        g = K.ConvGeom(B, H, H, C_, C_, 3, 3, 1, 1)
        x = torch.randn(B, H, H, C_, device=dev).to(dt)
        xa = torch.empty_like(x)
        w = (torch.randn(C_, 3, 3, C_, device=dev) * 0.05).to(dt)
        y = torch.empty_like(x)
        sc = torch.rand(C_, device=dev) + 0.5
        sh = torch.randn(C_, device=dev) * 0.1
        stats = torch.empty(math.ceil(B * H * H / 64) * 3 * C_, device=dev)
        wf = w.view(C_, -1)
        halo = (2256, C_ if C_ <= 128 else 128)
        gen = (-128, halo[1])   # the register-staged tile the prologue used before the HALO form
        cases = {
            "fwd generic+prologue": lambda: K.conv_fwd(x, wf, g, y, stats=stats, pro=(sc, sh), tile=gen),
            "bn_apply": lambda: K.bn_apply(x, sc, sh, xa),
            "fwd HALO (applied input)": lambda: K.conv_fwd(xa, wf, g, y, stats=stats, tile=halo),
        }
        dy = torch.randn_like(x)
        dx = torch.empty_like(x)
        cases["dgrad generic"] = lambda: K.conv_dgrad(dy, w, g, dx, tile=K.pick_tile(B * H * H, C_, 9 * C_))
        cases["dgrad HALO"] = lambda: K.conv_dgrad(dy, w, g, dx, tile=halo)
        res = {k: [] for k in cases}
        for _ in range(3):   # alternate the cases
            for k, fn in cases.items():
                res[k].append(timeit(fn, reps))
        for k, v in res.items():
            print(f"{name} {k:28s} {statistics.median(v):8.1f} us")


if __name__ == "__main__":
    main()
