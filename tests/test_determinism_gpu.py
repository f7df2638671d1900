"""every cross-workgroup reduction is a fixed-order slab reduction, so two identical
training runs are bit-identical (no float atomics anywhere in the step)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _run(steps=2):
    from pytorch_distributed_amd.data import SyntheticImageNet
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    torch.manual_seed(0)
    m = NativeResNet(build_model("resnet50"), device=DEV, image_size=64)
    opt = m.make_optimizer(lr=0.01)
    crit = m.make_criterion()
    gen = m.input_generator(SyntheticImageNet("train", image_size=64))
    for i in range(steps):
        x, y = gen(torch.arange(12) + 12 * i)
        opt.zero_grad()
        crit(m(x), y).backward()
        opt.step()
    torch.cuda.synchronize()
    return m.flat_params.clone(), m.flat_buffers.clone()


def test_bitwise_reproducible_training_steps():
    p1, b1 = _run()
    p2, b2 = _run()
    assert torch.equal(p1, p2)
    assert torch.equal(b1, b2)
