"""csrc/tapconv.hip: the tap-reuse 3x3/1/1 64 -> 64 conv forward (layer1 conv2) vs a PyTorch fp32
conv of the same operands, the generic implicit-GEMM tile, and exact sums of its own output."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("pro", [False, True])
@pytest.mark.parametrize("Nb,H", [(2, 56), (3, 16), (2, 32)])
def test_tapconv_fwd(Nb, H, pro, dtype):
    from pytorch_distributed_amd.ops import native_ops as K
    torch.manual_seed(5)
    C = 64
    x = (torch.randn(Nb, H, H, C, device=DEV) + 0.2).to(dtype)
    w = (torch.randn(C, 3, 3, C, device=DEV) / 24).to(dtype)          # OHWI
    g = K.ConvGeom(Nb, H, H, C, C, 3, 3, 1, 1)
    assert K.tapconv_supported(g, dtype), "the tap-reuse kernel must handle this geometry"
    sc = (torch.rand(C, device=DEV) + 0.5) if pro else None
    sh = (torch.randn(C, device=DEV) * 0.3) if pro else None
    xa = x.float()
    if pro:   # the kernel rounds the activation to the storage dtype while staging
        xa = torch.relu(xa * sc + sh).to(dtype).float()
    y_ref = F.conv2d(xa.permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1)
    y_ref = y_ref.permute(0, 2, 3, 1)
    M = Nb * H * H
    rows = K.tapconv_stats_rows(g)
    y = torch.full((Nb, H, H, C), float("nan"), device=DEV, dtype=dtype)
    stats = torch.full((M // rows * 3 * C,), float("nan"), device=DEV)
    p = (sc, sh) if pro else None
    w2 = w.view(C, -1)
    K.tapconv_fwd(x, w2, g, y, stats, pro=p)
    y2, st2 = torch.empty_like(y), torch.empty_like(stats)
    K.tapconv_fwd(x, w2, g, y2, st2, pro=p)
    yg = torch.empty_like(y)
    K.conv_fwd(x, w2, g, yg, tile=(-128, 64), pro=p)   # the generic register tile
    y3 = torch.empty_like(y)
    K.tapconv_fwd(x, w2, g, y3, pro=p)
    torch.cuda.synchronize()
    assert torch.equal(y, y2) and torch.equal(stats, st2)
    assert torch.equal(y, y3)
    assert rel_err(y, y_ref) < 1e-2
    assert (y.float() - yg.float()).abs().max().item() <= 2e-2 * y_ref.abs().max().item()
    st = K.stats_totals(stats, M, C, rows).float()
    yb = y.float().reshape(-1, C)
    torch.testing.assert_close(st[0], yb.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(st[1], (yb * yb).sum(0), rtol=1e-3, atol=1e-2)
