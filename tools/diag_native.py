"""Per-block divergence of the native engine vs the fp32 torch reference (and torch bf16 autocast
as a precision yardstick). Usage: python tools/diag_native.py [arch] [image] [batch]"""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.models import build_model  # noqa: E402
from pytorch_distributed_amd.models.native import NativeResNet  # noqa: E402


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    arch = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    image = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ref = build_model(arch)
    tm = copy.deepcopy(ref).to(dev).train()
    tb = copy.deepcopy(ref).to(dev).train()
    nm = NativeResNet(ref, device=dev, dtype=torch.bfloat16, image_size=image).train()
    x = torch.randn(B, 3, image, image, device=dev).to(torch.bfloat16).float()
    outs = {}

    def hook(name, store):
        def h(m, i, o):
            store[name] = o.detach()
        return h

    fo, bo = {}, {}
    for n, m in tm.named_modules():
        if n.count(".") == 1 and n.startswith("layer"):
            m.register_forward_hook(hook(n, fo))
    for n, m in tb.named_modules():
        if n.count(".") == 1 and n.startswith("layer"):
            m.register_forward_hook(hook(n, bo))
    lt = tm(x)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lb = tb(x)
    ln = nm.native_forward(x, train=True, save=True)
    sv = nm._fwd_ctx
    names = [b.name for b in nm.blocks]
    print("stem y0 (pre-bn) vs torch conv1:", rel(sv["y0"].permute(0, 3, 1, 2), tm.conv1(x)))
    for i, n in enumerate(names[:-1]):
        nat = sv["blocks"][i + 1]["x"].permute(0, 3, 1, 2)
        print(f"{n:12s} native {rel(nat, fo[n]):.4f}   torch-bf16 {rel(bo[n], fo[n]):.4f}")
    print("logits      native", rel(ln, lt), " torch-bf16", rel(lb, lt))


if __name__ == "__main__":
    main()
