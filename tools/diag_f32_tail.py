"""Compare the native exact-fp32 engine's per-block tail gradients (dz = dL/d(bn3(y)+shortcut)
after the ReLU mask) with float64 autograd, block by block (ResNet-18/50)."""
import copy, os, sys
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.models import build_model
from pytorch_distributed_amd.models.native import NativeResNet

arch = sys.argv[1] if len(sys.argv) > 1 else "resnet18"
DEV = torch.device("cuda", 0)
torch.manual_seed(0)
ref = build_model(arch, 1000)
t64 = copy.deepcopy(ref).double()
nm = NativeResNet(ref, device=DEV, dtype=torch.float32, image_size=64)
torch.manual_seed(1)
x = torch.randn(8, 3, 64, 64)
y = torch.randint(0, 1000, (8,))
# reference: gradient at each block's output pre-ReLU = grad of (out before relu)
pre_grads = {}
blocks = [b for li in range(1, 5) for b in getattr(t64, f"layer{li}")]
def mk_hook(i):
    def fwd_hook(mod, inp, out):
        out.register_hook(lambda g: pre_grads.__setitem__(("out", i), g))
    return fwd_hook
for i, b in enumerate(blocks):
    b.register_forward_hook(mk_hook(i))
t64.train(); nm.train()
l64 = t64(x.double())
F.cross_entropy(l64, y).backward()
# native: capture tails (dz tensors) and block outputs' input-gradient
caught = {}
orig = NativeResNet._block_backward
def wrapped(self, b, rec, tail, prev, acc):
    i = self.blocks.index(b)
    caught[("tail_in", i)] = tail[0].clone()          # dz of this block's tail (masked)
    r = orig(self, b, rec, tail, prev, acc)
    return r
NativeResNet._block_backward = wrapped
ln = nm(x.to(DEV))
nm.make_criterion()(ln, y.to(DEV)).backward()
torch.cuda.synchronize()
# reference dz of block i's tail = dL/d(block_out) * (block_out > 0)  (out is post-ReLU)
outs = {}
def cap(i):
    def h(mod, inp, out):
        outs[i] = out.detach()
    return h
t2 = copy.deepcopy(t64)
for i, b in enumerate([b for li in range(1, 5) for b in getattr(t2, f"layer{li}")]):
    b.register_forward_hook(cap(i))
t2.train(); t2(x.double())
for i in range(len(blocks) - 1, -1, -1):
    g = pre_grads[("out", i)] * (outs[i] > 0)
    gn = caught[("tail_in", i)].cpu().double().permute(0, 3, 1, 2)
    e = ((gn - g).norm() / g.norm()).item()
    print(f"block {i}: tail dz rel err {e:.2e}  (|g| {g.norm().item():.3e})")
# block-0 detail: where do native and reference differ?
g = pre_grads[("out", 0)] * (outs[0] > 0)
gn = caught[("tail_in", 0)].cpu().double().permute(0, 3, 1, 2)
d = (gn - g).abs()
flat = d.flatten()
top = torch.topk(flat, 10)
print("abs diff: max", flat.max().item(), "mean", flat.mean().item(), "n>1e-6:", int((flat > 1e-6).sum()),
      "n>1e-4:", int((flat > 1e-4).sum()), "of", flat.numel())
for v, idx in zip(top.values.tolist(), top.indices.tolist()):
    n, c, h, w = torch.unravel_index(torch.tensor(idx), g.shape)
    print(f"  ({int(n)},{int(c)},{int(h)},{int(w)}) diff {v:.3e} native {gn[n,c,h,w].item():.4e} ref {g[n,c,h,w].item():.4e} out_ref {outs[0][n,c,h,w].item():.3e}")
