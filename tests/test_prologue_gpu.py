"""Fused BN-apply+ReLU prologue of the conv (fwd A operand, wgrad B operand) == materialised path."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("k,stride", [(3, 1), (1, 1), (3, 2)])
def test_conv_prologue_matches_materialised(k, stride):
    from pytorch_distributed_amd.ops import native_ops as K
    dt = torch.bfloat16
    Nb, H, Cin, Cout = 2, 12, 64, 128
    torch.manual_seed(0)
    y = torch.randn(Nb, H, H, Cin, device=DEV).to(dt)
    sc = torch.rand(Cin, device=DEV) + 0.5
    sh = torch.randn(Cin, device=DEV) * 0.5
    a = torch.empty_like(y)
    K.bn_apply(y, sc, sh, a, relu=True)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, k, k, stride, k // 2)
    w = (torch.randn(Cout, k, k, Cin, device=DEV) * 0.05).to(dt)
    out_ref = torch.empty(Nb, g.Ho, g.Wo, Cout, device=DEV, dtype=dt)
    out = torch.empty_like(out_ref)
    K.conv_fwd(a, w.view(Cout, -1), g, out_ref)
    K.conv_fwd(y, w.view(Cout, -1), g, out, pro=(sc, sh))
    dy = torch.randn_like(out_ref)
    ws = K.Workspace(DEV)
    gw_ref = torch.zeros(Cout * k * k * Cin, device=DEV)
    gw = torch.zeros_like(gw_ref)
    K.conv_wgrad(dy, a, g, gw_ref, ws)
    K.conv_wgrad(dy, y, g, gw, ws, pro=(sc, sh))
    torch.cuda.synchronize()
    assert torch.equal(out, out_ref)          # identical rounding of the activation
    assert rel_err(gw, gw_ref) < 1e-6
