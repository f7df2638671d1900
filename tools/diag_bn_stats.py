"""Per-unit BatchNorm batch statistics of the native engine (in-launch finalize) against float64
statistics of the same model's conv outputs, for the exact-fp32 and bf16 engines.
Usage (GPU): python tools/diag_bn_stats.py [arch] [image] [batch]"""
import sys

import torch


def main():
    arch = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    sys.path.insert(0, ".")
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    dev = torch.device("cuda", 0)
    for dt in (torch.float32, torch.bfloat16):
        torch.manual_seed(0)
        nm = NativeResNet(build_model(arch), device=dev, dtype=dt, image_size=S)
        torch.manual_seed(1)
        x = torch.randn(B, 3, S, S)
        # capture every unit's conv output by hooking the native schedule's conv_fwd
        from pytorch_distributed_amd.ops import native_ops as K
        outs = []
        orig = K.conv_fwd

        def spy(xx, w, g, out, *a, **k):
            r = orig(xx, w, g, out, *a, **k)
            if k.get("bn") is not None:
                outs.append((out, k["bn"]))
            return r
        K.conv_fwd = spy
        try:
            nm.train()
            with torch.no_grad():
                nm.native_forward(x.to(dev), train=True, save=False)
            torch.cuda.synchronize()
        finally:
            K.conv_fwd = orig
        worst = []
        for y, bn in outs:
            C = y.shape[-1]
            yd = y.double().reshape(-1, C)
            mean, var = yd.mean(0), yd.var(0, unbiased=False)
            em = ((bn.mean.double() - mean).abs() / (var.sqrt() + 1e-12)).max().item()
            inv_ref = 1 / torch.sqrt(var + 1e-5)
            ei = ((bn.invstd.double() - inv_ref).abs() / inv_ref).max().item()
            worst.append((round(em, 9), round(ei, 9), yd.shape[0], C))
        print(dt, "units", len(worst), "max mean err (in std units)", max(w[0] for w in worst),
              "max invstd rel err", max(w[1] for w in worst), flush=True)
        for w in worst[-6:]:
            print("   ", w)


if __name__ == "__main__":
    main()
