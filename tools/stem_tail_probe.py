"""Stem-backward tail at the production shape (ResNet-50, batch 400, 224 px), kernel by kernel:
stem_bwd_reduce alone and beside layer1's tap-reuse weight gradient on the second stream (the
in-step neighbour), the stem weight gradient as WGRAD_BNA (today) and as the
plain dz^T x / y0^T x halves of the decomposed form.

    python tools/stem_tail_probe.py            (GPU; prints one line per measurement)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    from pytorch_distributed_amd.data import SyntheticImageNet
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    from pytorch_distributed_amd.ops import native_ops as K
    dev = torch.device("cuda", 0)
    Nb = int(os.environ.get("PROBE_NB", "400"))
    torch.manual_seed(0)
    m = NativeResNet(build_model("resnet50"), device=dev, image_size=224)
    gen = m.input_generator(SyntheticImageNet("train", image_size=224))
    x, _ = gen(torch.arange(Nb))
    m.native_forward(x, train=True, save=True)
    sv = m._fwd_ctx
    x0, y0, arg, st0 = sv["x0"], sv["y0"], sv["arg"], sv["stem_stats"]
    u = m.stem
    g0 = u.geom(Nb)
    ws, ws_w = m.ws, m.ws_w
    Ho = y0.shape[1] // 2
    dout = (torch.randn(Nb, Ho, Ho, y0.shape[3], device=dev) * 1e-3).to(y0.dtype)
    dout2 = (torch.randn(Nb, Ho, Ho, y0.shape[3], device=dev) * 1e-3).to(y0.dtype)
    dz0 = torch.empty_like(y0)
    torch.cuda.synchronize()

    def timed(fn, n=20, warm=3):
        for _ in range(warm):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(n)]
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
        return ts[len(ts) // 2]

    MB = 1e-6
    red = lambda: K.stem_bwd_reduce(ws, dout, arg, y0, st0[2], st0[3], dz0, dout2=dout2)
    mb_red = (dout.numel() * 2 * 2 + arg.numel() + y0.numel() * 2 * 2) * MB
    t = timed(red)
    print(f"stem_bwd_reduce alone        {t:8.1f} us  {mb_red / t:5.2f} TB/s ({mb_red:.0f} MB)")
    part, G, nq = red()
    k0 = m._stem_k
    K.bn_bwd_finish(ws, part, G, nq, y0, st0[0], st0[1], m.gamma(u), m.dgamma(u), m.dbeta(u),
                    dz0, None, k_out=k0)
    mb_x = x0.numel() * 2 * MB
    if K.wgrad_bna_ok(g0, Nb, y0.dtype):
        t = timed(lambda: K.conv_wgrad(dz0, x0, g0, m.stem_wgrad, ws, bna=(y0, k0)))
        mb = (2 * y0.numel() * 2) * MB + mb_x
        print(f"stem wgrad BNA (dz, y0, x0)  {t:8.1f} us  {mb / t:5.2f} TB/s")
    t = timed(lambda: K.conv_wgrad(dz0, x0, g0, m.stem_wgrad, ws))
    mb = y0.numel() * 2 * MB + mb_x
    print(f"stem wgrad plain (dz, x0)    {t:8.1f} us  {mb / t:5.2f} TB/s")

    # beside the tap-reuse wgrad of layer1.0.conv2 on the second stream
    b = m.blocks[0]
    uc = b.units[1]
    g = uc.geom(Nb)
    H = g.H
    dy = (torch.randn(Nb, H, H, uc.cout, device=dev) * 1e-3).to(y0.dtype)
    a = torch.randn(Nb, H, H, uc.conv.in_channels, device=dev).to(y0.dtype)
    side = torch.cuda.Stream(dev)
    tap = lambda: K.conv_wgrad(dy, a, g, m.wgrad_view(uc), ws_w)
    with torch.cuda.stream(side):
        t_tap = timed(tap)
    print(f"l1.0.conv2 wgrad alone       {t_tap:8.1f} us  (tap path: {K.wgrad_tap_ok(g, y0.dtype)})")
    ts = []
    for _ in range(10):
        torch.cuda.synchronize()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            tap()
        a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a_.record()
        red()
        b_.record()
        torch.cuda.synchronize()
        ts.append(a_.elapsed_time(b_) * 1e3)
    ts.sort()
    print(f"stem_bwd_reduce beside tap   {ts[len(ts) // 2]:8.1f} us")
    both = []
    for _ in range(10):
        torch.cuda.synchronize()
        a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a_.record()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            tap()
        red()
        torch.cuda.current_stream().wait_stream(side)
        b_.record()
        torch.cuda.synchronize()
        both.append(a_.elapsed_time(b_) * 1e3)
    both.sort()
    print(f"reduce || tap (span)         {both[len(both) // 2]:8.1f} us")
    print("stem_tail_probe: ok")


if __name__ == "__main__":
    main()
