"""A/B of the conv forward launcher of two kernel libraries, shape by shape, on one device.

    python tools/fwd_ab.py LIB_A LIB_B [--with-fin-a] [--with-fin-b]

Each library's ``pda_conv_fwd`` is called through its own ctypes binding (``--with-fin-X``: that
library's launcher takes a BnFin pointer before ``dt``, an intermediate round-2 ABI), with the same
operands, tile (ops.native_ops.pick_tile), BatchNorm partial statistics and operand prologue as in
the ResNet-50 step; the launches alternate A/B so clock drift hits both alike. Prints the median
microseconds per shape and the COUNT-weighted total (tools/conv_bench.py SHAPES / COUNT)."""
import ctypes as C
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402
from tools.conv_bench import COUNT, SHAPES  # noqa: E402


def bind(path, with_fin):
    lib = C.CDLL(path)
    f = lib.pda_conv_fwd
    V, I = C.c_void_p, C.c_int
    args = [C.POINTER(ext.ConvDesc), V, V, I, V, I, I, V, V, I, V, V]
    if with_fin:
        args.append(V)
    f.argtypes = args + [I, I, I, V]
    f.restype = C.c_int
    return f, with_fin


def main():
    a, b = sys.argv[1], sys.argv[2]
    fa = bind(a, "--with-fin-a" in sys.argv)
    fb = bind(b, "--with-fin-b" in sys.argv)
    B = int(os.environ.get("BATCH", "400"))
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    st = torch.cuda.current_stream().cuda_stream
    tot = {"A": 0.0, "B": 0.0}
    for name, H, Cin, Cout, k, s in SHAPES:
        g = K.ConvGeom(B, H, H, Cin, Cout, k, k, s, k // 2)
        M = B * g.Ho * g.Wo
        x = torch.randn(B, H, H, Cin, device=dev).to(dt)
        w = (torch.randn(Cout, k * k * Cin, device=dev) * 0.05).to(dt)
        y = torch.empty(M, Cout, device=dev, dtype=dt)
        stats = torch.empty(math.ceil(M / 64) * 3 * Cout, device=dev)
        sc = torch.rand(Cin, device=dev) + 0.5
        sh = torch.randn(Cin, device=dev) * 0.1
        bm, bn = K.pick_tile(M, Cout, w.shape[1])
        desc = g.desc()
        pro = (sc.data_ptr(), sh.data_ptr()) if k == 3 or Cin == Cout else (None, None)

        def call(fw):
            f, fin = fw
            args = [C.byref(desc), x.data_ptr(), w.data_ptr(), w.shape[1], y.data_ptr(), 0, Cout,
                    None, stats.data_ptr(), 0, pro[0], pro[1]]
            if fin:
                args.append(None)
            rc = f(*args, ext.DT[dt], bm, bn, st)
            assert rc == 0, rc

        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ta, tb = [], []
        for it in range(12):
            ev[0].record(); call(fa); ev[1].record()
            ev[2].record(); call(fb); ev[3].record()
            torch.cuda.synchronize()
            if it >= 2:
                ta.append(ev[0].elapsed_time(ev[1]) * 1e3)
                tb.append(ev[2].elapsed_time(ev[3]) * 1e3)
        ma, mb = statistics.median(ta), statistics.median(tb)
        tot["A"] += COUNT[name] * ma
        tot["B"] += COUNT[name] * mb
        print(f"{name:4s} {Cin:5d}->{Cout:5d} k{k} s{s} tile {bm:5d}x{bn:<4d} A {ma:8.1f} us  "
              f"B {mb:8.1f} us  {100 * (mb / ma - 1):+6.1f}%", flush=True)
    print(f"weighted total: A {tot['A']:.0f} us  B {tot['B']:.0f} us  "
          f"{100 * (tot['B'] / tot['A'] - 1):+.1f}%")


if __name__ == "__main__":
    main()
