"""T2 tier: every ResNet-50 conv shape (reduced batch) through
every compiled tile variant of the implicit-GEMM kernel, fwd / dgrad / wgrad, against a plain
PyTorch fp32 reference. The split-K weight-gradient path is exercised with several block
targets, so the parallel slab reduction sees 1..hundreds of splits."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"

SHAPES = [  # name, H, Cin, Cout, k, stride  
    ("C1", 56, 64, 64, 1, 1), ("C2", 56, 64, 64, 3, 1), ("C3", 56, 64, 256, 1, 1),
    ("C4", 56, 256, 64, 1, 1), ("C5", 56, 256, 128, 1, 1), ("C6", 56, 128, 128, 3, 2),
    ("C7", 28, 128, 512, 1, 1), ("C8", 56, 256, 512, 1, 2), ("C9", 28, 512, 128, 1, 1),
    ("C10", 28, 128, 128, 3, 1), ("C11", 28, 512, 256, 1, 1), ("C12", 28, 256, 256, 3, 2),
    ("C13", 14, 256, 1024, 1, 1), ("C14", 28, 512, 1024, 1, 2), ("C15", 14, 1024, 256, 1, 1),
    ("C16", 14, 256, 256, 3, 1), ("C17", 14, 1024, 512, 1, 1), ("C18", 14, 512, 512, 3, 2),
    ("C19", 7, 512, 2048, 1, 1), ("C20", 14, 1024, 2048, 1, 2), ("C21", 7, 2048, 512, 1, 1),
    ("C22", 7, 512, 512, 3, 1),
]
TILES = [(128, 128), (128, 64), (64, 128), (64, 64), (-128, 128), (-128, 64), (-64, 128)]
# LDS-DMA 8-wave tiles (bm = 1000 + rows): 16-bit only
DMA_TILES = [(1256, 128), (1128, 256), (1128, 128)]
# wgrad only: the 256-row single-stage tile and the 256x256 LDS-DMA tile (32 k per ring slot)
WGRAD_TILES = TILES + DMA_TILES + [(-256, 128), (1256, 256)]


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("shape", SHAPES, ids=[s[0] for s in SHAPES])
def test_resnet50_conv_shape_all_tiles(shape):
    from pytorch_distributed_amd.ops import ext
    ext.load(required=True)
    from pytorch_distributed_amd.ops import native_ops as K
    _, H, Cin, Cout, k, s = shape
    Nb, pad, dt = 2, k // 2, torch.bfloat16
    torch.manual_seed(1)
    x = (torch.randn(Nb, Cin, H, H, device=DEV) + 0.1).to(dt).float()
    w = (torch.randn(Cout, Cin, k, k, device=DEV) / math.sqrt(Cin * k * k)).to(dt).float()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y_ref = F.conv2d(xr, wr, stride=s, padding=pad)
    dy = torch.randn_like(y_ref).to(dt).float()
    y_ref.backward(dy)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, k, k, s, pad)
    x_nhwc = x.permute(0, 2, 3, 1).contiguous().to(dt)
    w_ohwi = w.permute(0, 2, 3, 1).contiguous().to(dt)
    dy_nhwc = dy.permute(0, 2, 3, 1).contiguous().to(dt)
    yr = y_ref.detach().permute(0, 2, 3, 1)
    dxr = xr.grad.permute(0, 2, 3, 1)
    dwr = wr.grad.permute(0, 2, 3, 1)
    ws = K.Workspace(DEV)
    M = Nb * g.Ho * g.Wo
    bad = []
    for t in WGRAD_TILES:
        if t not in TILES + DMA_TILES:   # wgrad-only tile
            for tb in (64, 512, 4096):
                dw = torch.full((Cout, k, k, Cin), float("nan"), device=DEV)
                K.conv_wgrad(dy_nhwc, x_nhwc, g, dw.view(-1), ws, tile=t, target_blocks=tb)
                torch.cuda.synchronize()
                e = rel_err(dw, dwr)
                if not e < 1e-2:
                    bad.append((t, f"wgrad/{tb}", e))
            continue
        y = torch.full((Nb, g.Ho, g.Wo, Cout), float("nan"), device=DEV, dtype=dt)
        stats = torch.zeros(math.ceil(M / 64) * 3 * Cout, device=DEV)
        K.conv_fwd(x_nhwc, w_ohwi.view(Cout, -1), g, y, stats=stats, tile=t)
        dx = torch.full((Nb, H, H, Cin), float("nan"), device=DEV, dtype=dt)
        K.conv_dgrad(dy_nhwc, w_ohwi, g, dx, tile=t)
        torch.cuda.synchronize()
        st = K.stats_totals(stats, M, Cout, t[0]).float()
        for name, e in (("fwd", rel_err(y, yr)), ("dgrad", rel_err(dx, dxr)),
                        ("stats", rel_err(st[0], y.float().reshape(-1, Cout).sum(0)))):
            if not e < 1e-2:
                bad.append((t, name, e))
        for tb in (64, 512, 4096):
            dw = torch.full((Cout, k, k, Cin), float("nan"), device=DEV)
            K.conv_wgrad(dy_nhwc, x_nhwc, g, dw.view(-1), ws, tile=t, target_blocks=tb)
            torch.cuda.synchronize()
            e = rel_err(dw, dwr)
            if not e < 1e-2:
                bad.append((t, f"wgrad/{tb}", e))
    assert not bad, bad


@pytest.mark.parametrize("shape", SHAPES, ids=[s[0] for s in SHAPES])
def test_resnet50_conv_shape_all_tiles_exact_f32(shape):
    """The exact-fp32 path (MFMA 16x16x4 f32) on every ResNet-50 shape and every f32 tile, against
    a float64 CPU reference: errors at fp32 rounding level."""
    from pytorch_distributed_amd.ops import ext
    ext.load(required=True)
    from pytorch_distributed_amd.ops import native_ops as K
    _, H, Cin, Cout, k, s = shape
    Nb, pad = 2, k // 2
    torch.manual_seed(1)
    x = torch.randn(Nb, Cin, H, H, dtype=torch.float64) + 0.1
    w = torch.randn(Cout, Cin, k, k, dtype=torch.float64) / math.sqrt(Cin * k * k)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y_ref = F.conv2d(xr, wr, stride=s, padding=pad)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, k, k, s, pad)
    x_nhwc = x.permute(0, 2, 3, 1).contiguous().float().to(DEV)
    w_ohwi = w.permute(0, 2, 3, 1).contiguous().float().to(DEV)
    dy_nhwc = dy.permute(0, 2, 3, 1).contiguous().float().to(DEV)
    yr = y_ref.detach().permute(0, 2, 3, 1)
    dxr = xr.grad.permute(0, 2, 3, 1)
    dwr = wr.grad.permute(0, 2, 3, 1)
    ws = K.Workspace(DEV)
    bad = []
    for t in TILES:
        y = torch.full((Nb, g.Ho, g.Wo, Cout), float("nan"), device=DEV)
        K.conv_fwd(x_nhwc, w_ohwi.view(Cout, -1), g, y, tile=t)
        dx = torch.full((Nb, H, H, Cin), float("nan"), device=DEV)
        K.conv_dgrad(dy_nhwc, w_ohwi, g, dx, tile=t)
        dw = torch.full((Cout, k, k, Cin), float("nan"), device=DEV)
        K.conv_wgrad(dy_nhwc, x_nhwc, g, dw.view(-1), ws, tile=t, target_blocks=512)
        torch.cuda.synchronize()
        for name, a, b in (("fwd", y, yr), ("dgrad", dx, dxr), ("wgrad", dw, dwr)):
            e = rel_err(a.cpu().double(), b)
            if not e < 1e-5:
                bad.append((t, name, e))
    assert not bad, bad


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("shape", [SHAPES[i] for i in (1, 5, 6, 11, 15, 17, 20, 21)],
                         ids=[SHAPES[i][0] for i in (1, 5, 6, 11, 15, 17, 20, 21)])
def test_dma_tiles_multi_tile(shape, dt):
    """The LDS-DMA tiles at a batch that gives many full M tiles (the 3-slot ring wraps, every
    slot is rewritten while other waves still compute): fwd + statistics, dgrad, wgrad vs fp32."""
    from pytorch_distributed_amd.ops import ext
    ext.load(required=True)
    from pytorch_distributed_amd.ops import native_ops as K
    _, H, Cin, Cout, k, s = shape
    Nb, pad = 24 if H <= 14 else 6, k // 2
    torch.manual_seed(2)
    x = (torch.randn(Nb, Cin, H, H, device=DEV) + 0.1).to(dt).float()
    w = (torch.randn(Cout, Cin, k, k, device=DEV) / math.sqrt(Cin * k * k)).to(dt).float()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y_ref = F.conv2d(xr, wr, stride=s, padding=pad)
    dy = torch.randn_like(y_ref).to(dt).float()
    y_ref.backward(dy)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, k, k, s, pad)
    x_nhwc = x.permute(0, 2, 3, 1).contiguous().to(dt)
    w_ohwi = w.permute(0, 2, 3, 1).contiguous().to(dt)
    dy_nhwc = dy.permute(0, 2, 3, 1).contiguous().to(dt)
    yr = y_ref.detach().permute(0, 2, 3, 1)
    ws = K.Workspace(DEV)
    M = Nb * g.Ho * g.Wo
    bad = []
    for t in DMA_TILES:
        y = torch.full((Nb, g.Ho, g.Wo, Cout), float("nan"), device=DEV, dtype=dt)
        stats = torch.zeros(math.ceil(M / 64) * 3 * Cout, device=DEV)
        K.conv_fwd(x_nhwc, w_ohwi.view(Cout, -1), g, y, stats=stats, tile=t)
        dx = torch.full((Nb, H, H, Cin), float("nan"), device=DEV, dtype=dt)
        K.conv_dgrad(dy_nhwc, w_ohwi, g, dx, tile=t)
        dw = torch.full((Cout, k, k, Cin), float("nan"), device=DEV)
        K.conv_wgrad(dy_nhwc, x_nhwc, g, dw.view(-1), ws, tile=t, target_blocks=512)
        torch.cuda.synchronize()
        st = K.stats_totals(stats, M, Cout, t[0]).float()
        for name, e in (("fwd", rel_err(y, yr)), ("dgrad", rel_err(dx, xr.grad.permute(0, 2, 3, 1))),
                        ("wgrad", rel_err(dw, wr.grad.permute(0, 2, 3, 1))),
                        ("stats", rel_err(st[0], y.float().reshape(-1, Cout).sum(0)))):
            if not e < 1e-2:
                bad.append((t, name, e))
    for tb in (64, 256, 1024):   # the 256x256 weight-gradient tile, several split-K depths
        dw = torch.full((Cout, k, k, Cin), float("nan"), device=DEV)
        K.conv_wgrad(dy_nhwc, x_nhwc, g, dw.view(-1), ws, tile=(1256, 256), target_blocks=tb)
        torch.cuda.synchronize()
        e = rel_err(dw, wr.grad.permute(0, 2, 3, 1))
        if not e < 1e-2:
            bad.append(((1256, 256), f"wgrad/{tb}", e))
    assert not bad, bad


HALO_TILES = [(2256, 128), (2256, 64)]   # tap-reuse tiles: 3x3 stride-1 fwd / dgrad only


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("shape,Nb", [(SHAPES[1], 3), (SHAPES[9], 5), (SHAPES[15], 9), (SHAPES[21], 13),
                                      (SHAPES[15], 1), (SHAPES[21], 2)],
                         ids=["C2", "C10", "C16", "C22", "C16-1img", "C22-2img"])
def test_halo_tiles(shape, Nb, dt):
    """The tap-reuse tiles (one input slab per 64-channel chunk serves all 9 taps, shifted
    fragment reads, out-of-image taps read a zero row): every image border, ragged last M tile,
    tiles spanning several images, fwd + statistics and dgrad (+ BN-backward epilogue) vs fp32."""
    from pytorch_distributed_amd.ops import ext
    ext.load(required=True)
    from pytorch_distributed_amd.ops import native_ops as K
    _, H, Cin, Cout, k, s = shape
    torch.manual_seed(3)
    x = (torch.randn(Nb, Cin, H, H, device=DEV) + 0.1).to(dt).float()
    w = (torch.randn(Cout, Cin, k, k, device=DEV) / math.sqrt(Cin * k * k)).to(dt).float()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y_ref = F.conv2d(xr, wr, stride=s, padding=1)
    dy = torch.randn_like(y_ref).to(dt).float()
    y_ref.backward(dy)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, k, k, s, 1)
    x_nhwc = x.permute(0, 2, 3, 1).contiguous().to(dt)
    w_ohwi = w.permute(0, 2, 3, 1).contiguous().to(dt)
    dy_nhwc = dy.permute(0, 2, 3, 1).contiguous().to(dt)
    M = Nb * H * H
    bad = []
    for t in HALO_TILES:
        y = torch.full((Nb, H, H, Cout), float("nan"), device=DEV, dtype=dt)
        stats = torch.zeros(math.ceil(M / 64) * 3 * Cout, device=DEV)
        K.conv_fwd(x_nhwc, w_ohwi.view(Cout, -1), g, y, stats=stats, tile=t)
        dx = torch.full((Nb, H, H, Cin), float("nan"), device=DEV, dtype=dt)
        K.conv_dgrad(dy_nhwc, w_ohwi, g, dx, tile=t)
        torch.cuda.synchronize()
        st = K.stats_totals(stats, M, Cout, t[0]).float()
        for name, e in (("fwd", rel_err(y, y_ref.detach().permute(0, 2, 3, 1))),
                        ("dgrad", rel_err(dx, xr.grad.permute(0, 2, 3, 1))),
                        ("stats", rel_err(st[0], y.float().reshape(-1, Cout).sum(0)))):
            if not e < 1e-2:
                bad.append((t, name, e))
    assert not bad, bad
