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


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("S", [32, 96, 224])
def test_stem_fwd_kernel(S, dtype):
    """csrc/stem.hip (LDS tap-reuse stem conv + shifted BN partials) vs the fp32 torch conv, the
    generic implicit-GEMM tile and exact sums of its own output; bitwise run-to-run."""
    from pytorch_distributed_amd.ops import native_ops as K
    Nb = 2
    torch.manual_seed(3)
    x = (torch.randn(Nb, 3, S, S, device=DEV) + 0.3).to(dtype).float()
    w = (torch.randn(64, 3, 7, 7, device=DEV) * 0.05).to(dtype).float()
    y_ref = F.conv2d(x, w, stride=2, padding=3).permute(0, 2, 3, 1)
    xs = torch.empty(Nb, S // 2, S // 2, 16, device=DEV, dtype=dtype)
    K.nchw_to_s2d(x, xs)
    packed = torch.empty(64, 256, device=DEV, dtype=dtype)
    K.pack_stem_s2d(w.permute(0, 2, 3, 1).contiguous(), packed)
    g = K.stem_s2d_geom(Nb, S)
    assert K.stem_fwd_ok(g, dtype), "the stem kernel must run for this geometry"
    M = Nb * g.Ho * g.Wo
    rows = K.stem_stats_rows(g)
    y = torch.full((Nb, g.Ho, g.Wo, 64), float("nan"), device=DEV, dtype=dtype)
    stats = torch.full((M // rows * 3 * 64,), float("nan"), device=DEV)
    K.stem_fwd(xs, packed, g, y, stats)
    y2 = torch.empty_like(y)
    stats2 = torch.empty_like(stats)
    K.stem_fwd(xs, packed, g, y2, stats2)
    yg = torch.empty_like(y)
    K.conv_fwd(xs, packed, g, yg, tile=(-128, 64))   # the generic register tile
    torch.cuda.synchronize()
    assert torch.equal(y, y2) and torch.equal(stats, stats2)
    assert rel_err(y, y_ref) < 1e-2
    assert (y.float() - yg.float()).abs().max().item() <= 2e-2 * y_ref.abs().max().item()
    st = K.stats_totals(stats, M, 64, rows).float()
    yb = y.float().reshape(-1, 64)
    torch.testing.assert_close(st[0], yb.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(st[1], (yb * yb).sum(0), rtol=1e-3, atol=1e-2)
    # no statistics: same output
    y3 = torch.empty_like(y)
    K.stem_fwd(xs, packed, g, y3)
    torch.cuda.synchronize()
    assert torch.equal(y, y3)


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
