"""Diagnose DP graph vs eager: compare both to a manual two-model reference per step."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.data import SyntheticImageNet
from pytorch_distributed_amd.models import build_model
from pytorch_distributed_amd.models.native import NativeResNet
from pytorch_distributed_amd.parallel import DataParallel

DEV = torch.device("cuda", 0)
torch.manual_seed(0)
sd = build_model("resnet18").state_dict()
def mk():
    r = build_model("resnet18"); r.load_state_dict(sd)
    return NativeResNet(r, device=DEV, image_size=64)
eager = DataParallel(mk(), device_ids=[0, 0])
graphed = DataParallel(mk(), device_ids=[0, 0])
gen = eager.module.input_generator(SyntheticImageNet("train", image_size=64))
crit = torch.nn.CrossEntropyLoss()
oe = eager.make_optimizer(lr=0.05, momentum=0.9, weight_decay=1e-4)
og = graphed.make_optimizer(lr=0.05, momentum=0.9, weight_decay=1e-4)
def rel(a, b):
    return ((a - b).norm() / (a.norm() + 1e-30)).item()
for step in range(4):
    x, y = gen(torch.arange(16) + 16 * step)
    oe.zero_grad()
    le = crit(eager(x), y); le.backward()
    torch.cuda.synchronize()
    ge0, ge1 = eager.module.flat_grad.clone(), eager.replicas[0].flat_grad.clone()
    lg = graphed.train_step(x, y, og)
    torch.cuda.synchronize()
    gg0, gg1 = graphed.module.flat_grad.clone(), graphed.replicas[0].flat_grad.clone()
    print(step, "loss", le.item(), lg.item(), "grad e0-g0", rel(ge0, gg0), "e0-e1", rel(ge0, ge1),
          "g0-g1", rel(gg0, gg1), "params", rel(eager.module.flat_params, graphed.module.flat_params),
          "buffers", rel(eager.module.flat_buffers, graphed.module.flat_buffers),
          "rep buffers e", rel(eager.module.flat_buffers, eager.replicas[0].flat_buffers),
          "rep buffers g", rel(graphed.module.flat_buffers, graphed.replicas[0].flat_buffers), flush=True)
    oe.step()
