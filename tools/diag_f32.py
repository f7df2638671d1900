"""Per-parameter gradient error of the native exact-fp32 engine and of torch fp32 (CPU), both
against float64 -- separates conditioning (both large) from a kernel bug (native alone large)."""
import copy, os, sys
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.models import build_model
from pytorch_distributed_amd.models.native import NativeResNet

arch = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
DEV = torch.device("cuda", 0)
torch.manual_seed(0)
ref = build_model(arch, 1000)
t64 = copy.deepcopy(ref).double()
t32 = copy.deepcopy(ref)
nm = NativeResNet(ref, device=DEV, dtype=torch.float32, image_size=64)
torch.manual_seed(1)
x = torch.randn(B, 3, 64, 64)
y = torch.randint(0, 1000, (B,))
for m in (t64, t32, nm):
    m.train()
l64 = t64(x.double()); l32 = t32(x); ln = nm(x.to(DEV))
F.cross_entropy(l64, y).backward(); F.cross_entropy(l32, y).backward()
nm.make_criterion()(ln, y.to(DEV)).backward()
torch.cuda.synchronize()
def re(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()
print("logits native", re(ln.cpu(), l64), "torch32", re(l32, l64))
p64 = dict(t64.named_parameters()); p32 = dict(t32.named_parameters())
for n, p in reversed(list(nm.named_parameters())):
    print(f"{n:40s} native {re(p.grad.cpu(), p64[n].grad):.2e}  torch32 {re(p32[n].grad, p64[n].grad):.2e}")
