"""HIP-graph capture of the native training step: replaying the captured step must reproduce the
eager step bit for bit (every kernel is deterministic -- no float atomics), for bf16 and for the
fp16 AMP path (device-side loss scaling), and an LR change must trigger a re-capture."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(dtype, graph, steps=4, lr_change_at=None):
    from pytorch_distributed_amd.models.native import NativeTrainer
    dev = torch.device("cuda", 0)
    tr = NativeTrainer("resnet50", 16, dtype, dev, image_size=64, graph=graph)
    losses = []
    for i in range(steps):
        if lr_change_at is not None and i == lr_change_at:
            tr.opt.param_groups[0]["lr"] = 0.01
        tr.step(i)
        losses.append(tr.last_loss())
    torch.cuda.synchronize()
    return tr, losses


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_graph_replay_matches_eager(dtype):
    te, le = _run(dtype, graph=False)
    tg, lg = _run(dtype, graph=True)
    assert tg.graphed.captures == 1
    assert le == lg, (le, lg)
    assert torch.equal(te.model.flat_params, tg.model.flat_params)
    assert torch.equal(te.opt.flat_mom, tg.opt.flat_mom)
    assert torch.equal(te.model.flat_buffers, tg.model.flat_buffers)   # BN running stats
    if dtype == torch.float16:
        assert te.scaler.get_scale() == tg.scaler.get_scale()


def test_graph_recaptures_on_lr_change():
    te, le = _run(torch.bfloat16, graph=False, steps=4, lr_change_at=2)
    tg, lg = _run(torch.bfloat16, graph=True, steps=4, lr_change_at=2)
    assert tg.graphed.captures == 2
    assert le == lg
    assert torch.equal(te.model.flat_params, tg.model.flat_params)
