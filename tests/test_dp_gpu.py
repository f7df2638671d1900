"""Native DataParallel semantics on one GPU: two replicas sharing cuda:0 (plain-copy sync path)
must produce the same update as one model on the concatenated batch."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_native_dataparallel_matches_single_model():
    from pytorch_distributed_amd.data import SyntheticImageNet
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    from pytorch_distributed_amd.parallel import DataParallel
    torch.manual_seed(0)
    ref = build_model("resnet18")
    sd = {k: v.clone() for k, v in ref.state_dict().items()}
    single = NativeResNet(ref, device=DEV, image_size=64)
    ref2 = build_model("resnet18")
    ref2.load_state_dict(sd)
    dp = DataParallel(NativeResNet(ref2, device=DEV, image_size=64), device_ids=[0, 0])
    gen = single.input_generator(SyntheticImageNet("train", image_size=64))
    x, y = gen(torch.arange(16))
    # BN statistics are per replica in DP (as in torch): compare against two half batches
    crit = torch.nn.CrossEntropyLoss()
    opt_dp = dp.make_optimizer(lr=0.05, momentum=0.9, weight_decay=1e-4)
    opt_dp.zero_grad()
    crit(dp(x), y).backward()
    torch.cuda.synchronize()
    g_dp = dp.module.flat_grad.clone()
    assert torch.equal(dp.module.flat_grad, dp.replicas[0].flat_grad)
    # reference: gradient of the mean loss over the global batch, each half with its own BN stats
    g_ref = torch.zeros_like(g_dp)
    for h in range(2):
        single.zero_grad_flat()
        out = single(x[h * 8:(h + 1) * 8])
        (crit(out, y[h * 8:(h + 1) * 8]) * 0.5).backward()
        g_ref += single.flat_grad
    err = ((g_dp - g_ref).norm() / g_ref.norm()).item()
    assert err < 1e-4, err
    opt_dp.step()
    torch.cuda.synchronize()
    assert torch.equal(dp.module.flat_params, dp.replicas[0].flat_params)
