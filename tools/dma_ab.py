"""A/B of conv kernel variants in ONE process (cdna_hip_programming.md §5.4 rule 24).

Build (CPU):  python tools/dma_ab.py build NAME [-DFLAG=V ...] [--full]
    -> pytorch_distributed_amd/_lib/ab/libconv_NAME.so (conv_gemm.hip only; without --full
       only the LDS-DMA instantiations: -DCONV_DMA_ONLY, a ~10 s build)
Run (GPU):    python tools/dma_ab.py run NAME[,NAME...] SHAPE:PASS:BM:BN [...] [--rounds R] [--reps N]
    times every (case, variant) interleaved over R rounds; prints the median and min (us, TF/s).
    NAME "main" = the in-tree libpda_kernels.so."""
import math
import os
import statistics
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def build(name, flags, full):
    from pytorch_distributed_amd import _build
    out = _build.OUT / "ab"
    out.mkdir(parents=True, exist_ok=True)
    obj = out / f"conv_{name}.o"
    extra = list(flags) + ([] if full else ["-DCONV_DMA_ONLY"])
    _build._compile(_build.CSRC / "conv_gemm.hip", obj, extra, verbose=True)
    lib = out / f"libconv_{name}.so"
    _build._link([obj], lib, [], verbose=False)
    obj.unlink()
    print(lib)


def run(names, cases, rounds, reps):
    import torch
    from pytorch_distributed_amd.ops import ext
    from pytorch_distributed_amd.ops import native_ops as K
    from tools.conv_bench import SHAPES
    libs = {}
    for n in names:
        ext._LIB = None
        ext.LIBPATH = (ext.LIBPATH.parent.parent / "_lib" / "libpda_kernels.so" if n == "main" else
                       ROOT / "pytorch_distributed_amd" / "_lib" / "ab" / f"libconv_{n}.so")
        libs[n] = ext.load(required=True)
    dev = torch.device("cuda", 0)
    B, dt = 400, torch.bfloat16
    ws = K.Workspace(dev)
    fns = []
    for c in cases:
        shape, ps, bm, bn = c.split(":")
        _, H, Cin, Cout, k, s = next(sh for sh in SHAPES if sh[0] == shape)
        g = K.ConvGeom(B, H, H, Cin, Cout, k, k, s, k // 2)
        x = torch.randn(B, H, H, Cin, device=dev).to(dt)
        w = (torch.randn(Cout, k, k, Cin, device=dev) * 0.05).to(dt)
        y = torch.empty(B, g.Ho, g.Wo, Cout, device=dev, dtype=dt)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        gw = torch.empty(Cout * k * k * Cin, device=dev)
        M = B * g.Ho * g.Wo
        stats = torch.empty(math.ceil(M / 64) * 3 * Cout, device=dev)
        t = (int(bm), int(bn))
        if ps == "fwd":
            f = (lambda x=x, w=w, g=g, y=y, st=stats, t=t, C=Cout:
                 K.conv_fwd(x, w.view(C, -1), g, y, stats=st, tile=t))
        elif ps == "dgrad":
            f = lambda dy=dy, w=w, g=g, dx=dx, t=t: K.conv_dgrad(dy, w, g, dx, tile=t)
        else:
            f = lambda dy=dy, x=x, g=g, gw=gw, t=t: K.conv_wgrad(dy, x, g, gw, ws, tile=t)
        fns.append((c, f, 2.0 * M * Cout * Cin * k * k))
    res = {(c, n): [] for c, _, _ in fns for n in names}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for r in range(rounds):
        for c, f, _ in fns:
            for n in names:
                ext._LIB = libs[n]
                try:
                    f()
                except RuntimeError:   # tile not built into this variant
                    res[(c, n)].append(float("inf"))
                    continue
                torch.cuda.synchronize()
                ev[0].record()
                for _ in range(reps):
                    f()
                ev[1].record()
                torch.cuda.synchronize()
                res[(c, n)].append(ev[0].elapsed_time(ev[1]) / reps * 1e3)
    for c, _, fl in fns:
        line = f"{c:22s}"
        for n in names:
            v = res[(c, n)]
            md = statistics.median(v)
            line += f"  {n}: {md:7.1f} (min {min(v):7.1f}) {fl / md / 1e6:5.0f}TF"
        print(line, flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        args = sys.argv[3:]
        build(sys.argv[2], [a for a in args if a.startswith("-D")], "--full" in args)
    else:
        a = sys.argv[2:]
        rounds = int(a[a.index("--rounds") + 1]) if "--rounds" in a else 5
        reps = int(a[a.index("--reps") + 1]) if "--reps" in a else 5
        pos = [x for i, x in enumerate(a) if not x.startswith("--") and (i == 0 or not a[i - 1].startswith("--"))]
        run(pos[0].split(","), pos[1:], rounds, reps)
