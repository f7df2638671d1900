"""The space-to-depth stem: 7x7/2/3 conv on RGB == 4x4/1/2 conv on the 2x2 s2d image."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("S", [32, 64])
def test_stem_s2d_fwd_wgrad(S):
    from pytorch_distributed_amd.ops import native_ops as K
    dt = torch.bfloat16
    Nb = 3
    torch.manual_seed(2)
    x = torch.randn(Nb, 3, S, S, device=DEV).to(dt).float()
    w = (torch.randn(64, 3, 7, 7, device=DEV) * 0.05).to(dt).float()
    wr = w.clone().requires_grad_(True)
    y_ref = F.conv2d(x, wr, stride=2, padding=3)
    xs = torch.empty(Nb, S // 2, S // 2, 16, device=DEV, dtype=dt)
    K.nchw_to_s2d(x, xs)
    packed = torch.empty(64, 256, device=DEV, dtype=dt)
    K.pack_stem_s2d(w.permute(0, 2, 3, 1).contiguous(), packed)
    g = K.stem_s2d_geom(Nb, S)
    y = torch.empty(Nb, S // 2, S // 2, 64, device=DEV, dtype=dt)
    K.conv_fwd(xs, packed, g, y)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref.permute(0, 2, 3, 1)) < 1e-2
    dy = torch.randn_like(y_ref).to(dt).float()
    y_ref.backward(dy)
    gp = torch.zeros(64 * 256, device=DEV)
    K.conv_wgrad(dy.permute(0, 2, 3, 1).contiguous().to(dt), xs, g, gp, K.Workspace(DEV))
    gw = torch.zeros(64, 7, 7, 3, device=DEV)
    K.stem_s2d_grad(gp, gw.view(-1))
    torch.cuda.synchronize()
    assert rel_err(gw, wr.grad.permute(0, 2, 3, 1)) < 1e-2


def test_synth_s2d_matches_torch_generator():
    from pytorch_distributed_amd.data.synthetic import synthetic_images
    from pytorch_distributed_amd.ops import native_ops as K
    ids = torch.tensor([3, 11, 500000], device=DEV)
    S = 32
    out = torch.empty(3, S // 2, S // 2, 16, device=DEV, dtype=torch.bfloat16)
    lab = torch.empty(3, dtype=torch.int64, device=DEV)
    keys = torch.empty(3, dtype=torch.int32, device=DEV)
    K.synth_batch_s2d(ids, 0, "val", 1000, S, out, lab, keys)
    xr, yr = synthetic_images(ids.cpu(), 0, "val", 1000, S)
    ref = torch.empty(3, S // 2, S // 2, 16, device=DEV, dtype=torch.bfloat16)
    K.nchw_to_s2d(xr.to(DEV), ref)
    torch.cuda.synchronize()
    assert torch.equal(lab.cpu(), yr)
    torch.testing.assert_close(out.float(), ref.float(), rtol=1e-2, atol=2e-2)
