"""Per-parameter gradient agreement of the native bf16 step vs torch fp32 (cudnn off) and torch bf16
autocast vs fp32, at a given batch / image size: which parameters carry the global gradient norm and
where the engines disagree (the smoke oracle's calibration). Usage: python tools/smoke_diag.py B S"""
import copy
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    from pytorch_distributed_amd.data.synthetic import synthetic_images
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ref = build_model("resnet50")
    x, y = synthetic_images(torch.arange(B), 0, "train", 1000, S, device=dev)
    x = x.to(torch.bfloat16).float()
    g = {}
    for mode in ("fp32", "bf16"):
        tm = copy.deepcopy(ref).to(dev).train()
        with torch.backends.cudnn.flags(enabled=False), \
                torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode == "bf16"):
            loss = F.cross_entropy(tm(x).float(), y)
            loss.backward()
        g[mode] = ({n: p.grad.float().clone() for n, p in tm.named_parameters()}, float(loss))
    nm = NativeResNet(ref, device=dev, dtype=torch.bfloat16, image_size=S).train()
    loss = nm.make_criterion()(nm(x), y)
    loss.backward()
    g["native"] = ({n: p.grad.float().clone() for n, p in nm.named_parameters()}, float(loss))
    torch.cuda.synchronize()
    gt = g["fp32"][0]
    norm = {k: math.sqrt(sum(float(v.pow(2).sum()) for v in g[k][0].values())) for k in g}
    print(f"B={B} S={S} loss fp32 {g['fp32'][1]:.5f} bf16 {g['bf16'][1]:.5f} native {g['native'][1]:.5f}")
    print("grad norm", {k: round(v, 4) for k, v in norm.items()})
    rows = []
    for n, t in gt.items():
        tn = float(t.norm())
        eb = float((g["bf16"][0][n] - t).norm()) / (tn + 1e-12)
        en = float((g["native"][0][n] - t).norm()) / (tn + 1e-12)
        rows.append((tn, n, en, eb, float(g["native"][0][n].norm())))
    rows.sort(reverse=True)
    print("top parameters by fp32 gradient norm: name, |g| fp32, |g| native, rel err native, rel err bf16")
    for tn, n, en, eb, nn_ in rows[:15]:
        print(f"  {n:40s} {tn:10.4f} {nn_:10.4f} {en:8.4f} {eb:8.4f}")
    worst = sorted(rows, key=lambda r: -(r[2] / (r[3] + 1e-3)))[:10]
    print("worst native/bf16 error ratio:")
    for tn, n, en, eb, nn_ in worst:
        print(f"  {n:40s} {tn:10.4f} {en:8.4f} {eb:8.4f}")


if __name__ == "__main__":
    main()
