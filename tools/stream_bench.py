"""Isolated timing of the 16-bit BatchNorm streaming passes (csrc/bn.hip) on the ResNet-50 batch-400
activation shapes, for several streaming-kernel configurations (pda_set_stream_cfg: chunks per
thread per trip U, nontemporal policy NTM, grid cap):

  bwd  bn_bwd_apply (dz read back): dy = k1*dz + k2*y + k3   -- 2 reads + 1 write per element
  fwd  bn_apply mode 0 + ReLU + bitmask                       -- 1 read + 1 write (+ 1/16 mask)
  res  bn_apply mode 1 (+ residual) + ReLU + bitmask          -- 2 reads + 1 write

Prints us per launch and TB/s per shape, and the per-step weighted totals.

    python tools/stream_bench.py [U,NTM,CAP ...]     (default: 0,0,8192 1,0,8192 ... ; 'auto' = the
    size-dependent default policy)"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402

B = 400
# (rows, C, BN layers of this shape per step) -- every BN has one backward apply
SHAPES = [(B * 56 * 56, 64, 6), (B * 56 * 56, 256, 4), (B * 56 * 56, 128, 1),
          (B * 28 * 28, 128, 7), (B * 28 * 28, 512, 5), (B * 28 * 28, 256, 1), (B * 14 * 14, 256, 11),
          (B * 14 * 14, 1024, 7), (B * 14 * 14, 512, 1), (B * 7 * 7, 512, 5), (B * 7 * 7, 2048, 4)]


def timeit(fn, inner=10, outer=5):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(outer):
        ev[0].record()
        for _ in range(inner):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e3 / inner)
    return statistics.median(ts)


def main():
    L = ext.lib()
    dev = torch.device("cuda", 0)
    cfgs = sys.argv[1:] or ["0,0,8192", "1,0,8192", "2,0,8192", "4,0,8192", "2,1,8192", "2,2,8192",
                            "2,3,8192", "2,0,4096", "2,0,16384", "4,3,16384"]
    bufs = {}
    ref = {}
    for cfg in cfgs:
        u, ntm, cap = (-1, 3, 16384) if cfg == "auto" else (int(v) for v in cfg.split(","))
        L.pda_set_stream_cfg(u, ntm, cap, 100)
        tot = {"bwd": 0.0, "fwd": 0.0, "res": 0.0}
        lines = []
        for M, C_, n in SHAPES:
            key = (M, C_)
            if key not in bufs:
                g = torch.Generator(device=dev).manual_seed(M + C_)
                mk = lambda: torch.randn(M, C_, device=dev, generator=g).to(torch.bfloat16)  # noqa: E731
                bufs[key] = (mk(), mk(), torch.empty(M, C_, device=dev, dtype=torch.bfloat16),
                             torch.randn(6 * C_, device=dev, generator=g),
                             torch.empty(M * C_ // 8, device=dev, dtype=torch.uint8))
            dz, y, out, k, mask = bufs[key]
            a = K.BwdArgs(None, None, None, 0, K.ptr(y), None, None, None, None, None, 1, None, None,
                          2, M, C_)
            st = K.stream(dev)

            def bwd():
                K.check(L.pda_bn_bwd_apply(ext.C.byref(a), K.ptr(dz), K.ptr(y), K.ptr(k[0:C_]),
                                           K.ptr(k[C_:2 * C_]), K.ptr(k[2 * C_:3 * C_]), K.ptr(out), 1,
                                           st), "bn_bwd_apply")

            def fwd():
                K.bn_apply(y, k[0:C_], k[C_:2 * C_], out, mask=mask)

            def res():
                K.bn_apply(y, k[0:C_], k[C_:2 * C_], out, res=dz, mask=mask)

            nbytes = M * C_ * 2
            r = {}
            for name, fn, mult in (("bwd", bwd, 3), ("fwd", fwd, 2 + 1 / 16), ("res", res, 3 + 1 / 16)):
                fn()
                torch.cuda.synchronize()
                chk = out.float().sum().item()
                if (key, name) in ref:
                    assert abs(chk - ref[(key, name)]) <= 1e-3 * max(1.0, abs(ref[(key, name)])), \
                        (cfg, key, name, chk, ref[(key, name)])
                else:
                    ref[(key, name)] = chk
                t = timeit(fn)
                r[name] = (t, nbytes * mult / t / 1e6)
                tot[name] += n * t
            lines.append(f"  M {M:8d} C {C_:5d} x{n:2d}  " + "  ".join(
                f"{nm} {t:7.1f} us {bw:4.2f} TB/s" for nm, (t, bw) in r.items()))
        print(f"cfg U,NTM,CAP = {cfg}: weighted/step  bwd {tot['bwd']:.0f} us  fwd(x n) "
              f"{tot['fwd']:.0f} us  res(x n) {tot['res']:.0f} us", flush=True)
        for ln in lines:
            print(ln)
    L.pda_set_stream_cfg(*ext.stream_cfg())


if __name__ == "__main__":
    main()
