"""T2 tier: numerics of every gfx950 kernel against plain PyTorch fp32 references.

Inputs are asymmetric random data rounded to the kernel's 16-bit dtype first, so the
reference sees exactly the kernel's inputs; tolerances are relative to the output scale.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _k():
    from pytorch_distributed_amd.ops import ext
    ext.load(required=True)
    from pytorch_distributed_amd.ops import native_ops as K
    return K


def rel_err(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


CONV_CASES = [
    # Nb, H, Cin, Cout, k, stride
    (2, 8, 64, 64, 1, 1),
    (2, 8, 64, 128, 3, 1),
    (3, 9, 64, 64, 3, 1),       # ragged M
    (2, 8, 128, 64, 3, 2),
    (2, 8, 64, 256, 1, 2),
    (2, 14, 256, 128, 1, 1),
    (1, 7, 512, 2048, 1, 1),
    (4, 4, 1024, 256, 1, 1),
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(case, dtype):
    K = _k()
    Nb, H, Cin, Cout, k, s = case
    pad = k // 2
    torch.manual_seed(0)
    x = (torch.randn(Nb, Cin, H, H, device=DEV) + 0.1).to(dtype).float()
    w = (torch.randn(Cout, Cin, k, k, device=DEV) / math.sqrt(Cin * k * k)).to(dtype).float()
    y_ref = F.conv2d(x, w, stride=s, padding=pad)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, k, k, s, pad)
    x_nhwc = x.permute(0, 2, 3, 1).contiguous().to(dtype)
    w_ohwi = w.permute(0, 2, 3, 1).contiguous().to(dtype)
    y = torch.empty(Nb, g.Ho, g.Wo, Cout, device=DEV, dtype=dtype)
    M = Nb * g.Ho * g.Wo
    tile = K.fwd_tile(g, Nb, dtype)   # the default tile conv_fwd launches (DMA / HALO included)
    T = K.stats_tiles(M, Cout, tile)
    stats = torch.zeros(T * 3 * Cout, device=DEV)
    K.conv_fwd(x_nhwc, w_ohwi.view(Cout, -1), g, y, stats=stats)
    torch.cuda.synchronize()
    yr = y_ref.permute(0, 2, 3, 1)
    assert rel_err(y, yr) < 1e-2
    st = K.stats_totals(stats, M, Cout, tile[0]).float()
    yb = y.float().reshape(-1, Cout)
    torch.testing.assert_close(st[0], yb.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(st[1], (yb * yb).sum(0), rtol=1e-3, atol=1e-2)
    # backward
    dy = torch.randn_like(y_ref).to(dtype).float()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    F.conv2d(xr, wr, stride=s, padding=pad).backward(dy)
    dy_nhwc = dy.permute(0, 2, 3, 1).contiguous().to(dtype)
    dx = torch.full((Nb, H, H, Cin), float("nan"), device=DEV, dtype=dtype)
    K.conv_dgrad(dy_nhwc, w_ohwi, g, dx)
    ws = K.Workspace(DEV)
    dw = torch.zeros(Cout, k, k, Cin, device=DEV)
    K.conv_wgrad(dy_nhwc, x_nhwc, g, dw.view(-1), ws)
    torch.cuda.synchronize()
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2
    assert rel_err(dw, wr.grad.permute(0, 2, 3, 1)) < 1e-2


def test_conv_stem_padded_cin():
    K = _k()
    dtype = torch.bfloat16
    Nb, H = 2, 32
    torch.manual_seed(1)
    x = torch.randn(Nb, 3, H, H, device=DEV).to(dtype).float()
    w = (torch.randn(64, 3, 7, 7, device=DEV) * 0.05).to(dtype).float()
    y_ref = F.conv2d(x, w, stride=2, padding=3)
    x8 = torch.zeros(Nb, H, H, 8, device=DEV, dtype=dtype)
    x8[..., :3] = x.permute(0, 2, 3, 1).to(dtype)
    packed = torch.zeros(64, 448, device=DEV, dtype=dtype)
    K.pack_stem(w.permute(0, 2, 3, 1).contiguous(), packed)
    g = K.ConvGeom(Nb, H, H, 8, 64, 7, 7, 2, 3)
    y = torch.empty(Nb, g.Ho, g.Wo, 64, device=DEV, dtype=dtype)
    K.conv_fwd(x8, packed, g, y)
    dy = torch.randn_like(y_ref).to(dtype).float()
    wr = w.clone().requires_grad_(True)
    F.conv2d(x, wr, stride=2, padding=3).backward(dy)
    dw = torch.zeros(64, 7, 7, 3, device=DEV)
    K.conv_wgrad(dy.permute(0, 2, 3, 1).contiguous().to(dtype), x8, g, dw.view(-1), K.Workspace(DEV),
                 cin_real=3)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref.permute(0, 2, 3, 1)) < 1e-2
    assert rel_err(dw, wr.grad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("tile", [None, (-64, 128), (-64, 256)])
@pytest.mark.parametrize("Cout,Cin,k,H", [(64, 64, 3, 9), (64, 16, 4, 11), (64, 16, 4, 60)])
def test_conv_wgrad_bna_matches_applied(Cout, Cin, k, H, tile):
    """WGRAD_BNA (the stem wgrad forming dY = k1*dz + k2*y + k3 while staging) against the unfused
    path (dY materialised in bf16, plain wgrad) and against the fp32 PyTorch weight gradient of the
    same dY; ragged row counts check that padding rows contribute 0, not k3; H = 60 runs split-K."""
    K = _k()
    dtype = torch.bfloat16
    Nb = 3
    torch.manual_seed(Cout + k)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, k, k, 1, k // 2 if k != 4 else 0)
    if not K.wgrad_bna_ok(g, Nb, dtype):
        pytest.skip("tile not built for WGRAD_BNA")
    x = torch.randn(Nb, H, H, Cin, device=DEV).to(dtype)
    dz = torch.randn(Nb, g.Ho, g.Wo, Cout, device=DEV).to(dtype)
    y = (torch.randn(Nb, g.Ho, g.Wo, Cout, device=DEV) * 2 + 1).to(dtype)
    kk = torch.randn(3 * Cout, device=DEV)
    ws = K.Workspace(DEV)
    dw_f = torch.zeros(Cout, k, k, Cin, device=DEV)
    K.conv_wgrad(dz, x, g, dw_f.view(-1), ws, bna=(y, kk), tile=tile)
    # the kernels' fma chain fma(k1, dz, fma(k2, y, k3)), in f64 then rounded once to f32
    dy = (kk[:Cout].double() * dz.double() + (kk[Cout:2 * Cout].double() * y.double()
                                              + kk[2 * Cout:].double()).float().double()).float().to(dtype)
    dw_u = torch.zeros_like(dw_f)
    K.conv_wgrad(dy, x, g, dw_u.view(-1), ws)
    torch.cuda.synchronize()
    assert rel_err(dw_f, dw_u) < 2e-3
    wr = torch.zeros(Cout, Cin, k, k, device=DEV, requires_grad=True)
    out = F.conv2d(x.permute(0, 3, 1, 2).float(), wr, stride=1, padding=g.pad)
    out.backward(dy.permute(0, 3, 1, 2).float())
    assert rel_err(dw_f, wr.grad.permute(0, 2, 3, 1)) < 1e-2


def test_fc_as_conv():
    K = _k()
    dtype = torch.bfloat16
    B, Fd, Cls, rows = 5, 256, 100, 128
    x = torch.randn(B, Fd, device=DEV).to(dtype)
    w = torch.zeros(rows, Fd, device=DEV, dtype=dtype)
    w[:Cls] = (torch.randn(Cls, Fd, device=DEV) * 0.05).to(dtype)
    b = torch.randn(Cls, device=DEV)
    out = torch.empty(B, Cls, device=DEV)
    g = K.ConvGeom(B, 1, 1, Fd, Cls, 1, 1, 1, 0)
    K.conv_fwd(x, w, g, out, bias=b)
    torch.cuda.synchronize()
    ref = x.float() @ w[:Cls].float().t() + b
    assert rel_err(out, ref) < 1e-2


def _bn_ref(y, gamma, beta, eps=1e-5):
    mean = y.mean((0, 1, 2))
    var = y.var((0, 1, 2), unbiased=False)
    return mean, var, (y - mean) / torch.sqrt(var + eps) * gamma + beta


def test_bn_forward_finalize_apply():
    """bn_finalize_tot (the SyncBatchNorm path: f64 totals -> coefficients + running stats) and
    bn_apply against the plain PyTorch fp32 BatchNorm."""
    K = _k()
    dtype = torch.bfloat16
    N, H, C = 4, 6, 128
    y = (torch.randn(N, H, H, C, device=DEV) * 2 + 0.5).to(dtype)
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV)
    yd = y.double().reshape(-1, C)
    rows = yd.shape[0]
    tot = torch.stack([yd.sum(0), (yd * yd).sum(0)]).contiguous()
    st = torch.zeros(4, C, device=DEV)
    rm = torch.zeros(C, device=DEV)
    rv = torch.ones(C, device=DEV)
    nbt = torch.zeros(1, dtype=torch.int64, device=DEV)
    bn = K.BnStats(None, gamma, beta, 1e-5, 0.1, st[0], st[1], st[2], st[3], rm, rv, nbt)
    K.bn_finalize_tot(tot, C, rows, bn)
    out = torch.empty_like(y)
    K.bn_apply(y, st[2], st[3], out, relu=True)
    torch.cuda.synchronize()
    mean, var, ref = _bn_ref(y.float(), gamma, beta)
    torch.testing.assert_close(st[0], mean, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(st[1], 1 / torch.sqrt(var + 1e-5), rtol=1e-4, atol=1e-4)
    assert rel_err(out, torch.relu(ref)) < 1e-2
    torch.testing.assert_close(rm, 0.1 * mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rv, 0.9 + 0.1 * var * rows / (rows - 1), rtol=1e-4, atol=1e-5)
    assert int(nbt.item()) == 1


@pytest.mark.parametrize("cfg", [(0, 0, 8192, 100), (1, 0, 8192, 100), (2, 0, 8192, 100),
                                 (4, 3, 8192, 100), (2, 3, 7, 100), (4, 1, 3, 100), (-1, 3, 16384, 0),
                                 (4, 5, 8192, 100), (-1, 5, 7, 0)])
@pytest.mark.parametrize("C", [64, 256, 2048])
def test_bn_streaming_apply_configs(cfg, C):
    """bn_apply (modes 0/1/2 + ReLU bitmask) and bn_bwd_apply (dz read back) under every streaming
    configuration (chunks per thread U, memory policy -- nontemporal / write-through stores --,
    grid cap -- small caps force many trips and the remainder loop; -1 = the auto policy with its
    size threshold at 0) against plain PyTorch fp32 on the same bf16 inputs."""
    K = _k()
    from pytorch_distributed_amd.ops import ext
    L = ext.lib()
    rows = 1237 * 8   # ragged against U * stride
    g = torch.Generator(device=DEV).manual_seed(C)
    mk = lambda: torch.randn(rows, C, device=DEV, generator=g).to(torch.bfloat16)  # noqa: E731
    y, r, y2 = mk(), mk(), mk()
    sc, sh, sc2, sh2, k3 = (torch.randn(C, device=DEV, generator=g) for _ in range(5))
    out = torch.empty_like(y)
    mask = torch.empty(rows * C // 8, dtype=torch.uint8, device=DEV)
    bit = 1 << torch.arange(8, device=DEV)
    try:
        L.pda_set_stream_cfg(*cfg)
        for mode in (0, 1, 2):
            ref = y.float() * sc + sh
            if mode == 1:
                ref = ref + r.float()
            if mode == 2:
                ref = ref + y2.float() * sc2 + sh2
            ref = torch.relu(ref)
            K.bn_apply(y, sc, sh, out, res=r if mode == 1 else None, y2=y2 if mode == 2 else None,
                       scale2=sc2 if mode == 2 else None, shift2=sh2 if mode == 2 else None, mask=mask)
            torch.cuda.synchronize()
            torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-2)
            want = ((out.float().reshape(-1, 8) > 0).int() * bit).sum(1).to(torch.uint8)
            assert torch.equal(mask, want), (cfg, mode)
        a = K.BwdArgs(None, None, None, 0, K.ptr(y), None, None, None, None, None, 1, None, None, 2,
                      rows, C)
        K.check(L.pda_bn_bwd_apply(ext.C.byref(a), K.ptr(r), K.ptr(y), K.ptr(sc), K.ptr(sh), K.ptr(k3),
                                   K.ptr(out), 1, K.stream(torch.device(DEV))), "bn_bwd_apply")
        torch.cuda.synchronize()
        torch.testing.assert_close(out.float(), sc * r.float() + sh * y.float() + k3, rtol=1e-2,
                                   atol=2e-2)
    finally:
        L.pda_set_stream_cfg(*ext.stream_cfg())


def _conv_bn(K, x_nhwc, w2d, g, dtype, gamma, beta, tile=None, ws=None):
    ws = ws or K.Workspace(DEV)
    C = g.Cout
    y = torch.empty(x_nhwc.shape[0], g.Ho, g.Wo, C, device=DEV, dtype=dtype)
    st = torch.zeros(4, C, device=DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    nbt = torch.zeros(1, dtype=torch.int64, device=DEV)
    bn = K.BnStats(ws, gamma, beta, 1e-5, 0.1, st[0], st[1], st[2], st[3], rm, rv, nbt)
    K.conv_fwd(x_nhwc, w2d, g, y, bn=bn, tile=tile)
    return y, st, rm, rv, nbt, ws


@pytest.mark.parametrize("tile", [None, (-128, 128), (128, 64), (64, 128), (-128, 64)])
def test_conv_fwd_bn_finalize(tile):
    """BatchNorm statistics of the conv forward (shifted per-tile partials in the conv epilogue,
    then one launch: f64 slabs per block + last-arriver combine and finalize): mean / invstd /
    scale / shift / running stats / counter against float64 statistics of the stored output, on a
    ragged shape with several column tiles; bit-identical on a second launch (fixed summation
    order), arrival counters left at zero."""
    K = _k()
    dtype = torch.bfloat16
    torch.manual_seed(5)
    Nb, H, Cin, Cout = 7, 29, 64, 192
    g = K.ConvGeom(Nb, H, H, Cin, Cout, 3, 3, 1, 1)
    x = (torch.randn(Nb, H, H, Cin, device=DEV) + 0.2).to(dtype)
    w = (torch.randn(Cout, 3, 3, Cin, device=DEV) / 24).to(dtype)
    gamma, beta = torch.rand(Cout, device=DEV) + 0.5, torch.randn(Cout, device=DEV)
    y, st, rm, rv, nbt, ws = _conv_bn(K, x, w.view(Cout, -1), g, dtype, gamma, beta, tile)
    y2, st2, _, _, _, _ = _conv_bn(K, x, w.view(Cout, -1), g, dtype, gamma, beta, tile, ws)
    torch.cuda.synchronize()
    yd = y.double().reshape(-1, Cout)
    n = yd.shape[0]
    mean, var = yd.mean(0), yd.var(0, unbiased=False)
    torch.testing.assert_close(st[0].double(), mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(st[1].double(), 1 / torch.sqrt(var + 1e-5), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(st[2], gamma * st[1])
    torch.testing.assert_close(st[3], beta - st[0] * st[2])
    torch.testing.assert_close(rm.double(), 0.1 * mean, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(rv.double(), 0.9 + 0.1 * var * n / (n - 1), rtol=1e-5, atol=1e-7)
    assert int(nbt.item()) == 1
    assert torch.equal(y, y2) and torch.equal(st, st2)
    assert int(ws.counters(64).abs().sum().item()) == 0


class _DoublingComm:
    """Stand-in SyncBatchNorm communicator of two identical ranks: all_reduce doubles."""
    world_size = 2

    def all_reduce(self, t):
        t.mul_(2)


@pytest.mark.parametrize("sync", [False, True])
@pytest.mark.parametrize("C,T", [(64, 3), (192, 700), (512, 97), (1028, 40), (2048, 600)])
def test_bn_finalize_partials_channel_widths(C, T, sync):
    """The forward finalize (one launch: f64 slabs per (tile range, 256-channel group) block, the
    group's last arriver combines and finalizes) on synthetic shifted partials part[T][3][C] for
    every channel-width regime of its (channel quad x slab lane) decomposition -- several groups,
    a ragged last group (C = 1028), a ragged last tile -- against a float64 combination; ``sync``:
    the SyncBatchNorm path (f64 totals -> all-reduce -> finalize) with two identical ranks."""
    K = _k()
    torch.manual_seed(C + T)
    bm = 128
    M = T * bm - 37
    rows = torch.full((T,), float(bm), dtype=torch.float64)
    rows[-1] = M - (T - 1) * bm
    shift = torch.randn(T, C, dtype=torch.float64) * 3
    s1 = torch.randn(T, C, dtype=torch.float64) * 5
    s2 = torch.rand(T, C, dtype=torch.float64) * 200 + s1 ** 2 / rows[:, None]
    part = torch.stack([s1, s2, shift], 1).float()
    p64 = part.double()
    r = rows[:, None]
    tot1 = (r * p64[:, 2] + p64[:, 0]).sum(0)
    tot2 = (p64[:, 1] + p64[:, 2] * (2 * p64[:, 0] + r * p64[:, 2])).sum(0)
    mean = tot1 / M
    var = (tot2 / M - mean ** 2).clamp_min(0)
    ws = K.Workspace(DEV)
    if sync:
        ws.sync_comm = _DoublingComm()
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    st = torch.zeros(4, C, device=DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    nbt = torch.zeros(1, dtype=torch.long, device=DEV)
    bn = K.BnStats(ws, gamma, beta, 1e-5, 0.1, st[0], st[1], st[2], st[3], rm, rv, nbt,
                   update_running=True)
    K.bn_finalize_partials(part.to(DEV).contiguous(), T, C, bm, M, bn)
    torch.cuda.synchronize()
    n = M * (2 if sync else 1)
    torch.testing.assert_close(st[0].double().cpu(), mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(st[1].double().cpu(), 1 / torch.sqrt(var + 1e-5), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv.double().cpu(), 0.9 + 0.1 * var * n / (n - 1), rtol=1e-5, atol=1e-6)
    assert int(nbt.item()) == 1
    assert int(ws.counters(16).abs().sum().item()) == 0


@pytest.mark.parametrize("dtype,std", [(torch.float32, 0.01), (torch.bfloat16, 0.08)])
def test_bn_statistics_large_offset_layer1_scale(dtype, std):
    """Layer-1 scale (1.25 M rows x 64 channels, batch 400 at 56x56) with mean ~10 and std ~0.01
    (bf16: 0.08, so the stored values -- 1/16 apart at 10 -- still vary): E[y^2] - E[y]^2 from
    f32 partial sums would cancel catastrophically; the shifted per-tile sums + f64 combination
    must match float64 statistics of the stored output."""
    K = _k()
    torch.manual_seed(11)
    Nb, H, Cin, Cout = 400, 56, 64, 64
    g = K.ConvGeom(Nb, H, H, Cin, Cout, 1, 1, 1, 0)
    x = torch.randn(Nb, H, H, Cin, device=DEV)
    x[..., 0] = 1.0                                  # constant channel carries the offset
    w = torch.randn(Cout, Cin, device=DEV) * std / 8
    w[:, 0] = 10.0 + torch.rand(Cout, device=DEV)    # y_c ~ 10..11 + N(0, std^2)
    gamma, beta = torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV)
    y, st, rm, rv, nbt, _ = _conv_bn(K, x.to(dtype), w.to(dtype), g, dtype, gamma, beta)
    torch.cuda.synchronize()
    yd = y.double().reshape(-1, Cout)
    mean, var = yd.mean(0), yd.var(0, unbiased=False)
    assert float(var.min()) > 0
    got_var = 1.0 / st[1].double() ** 2 - 1e-5
    torch.testing.assert_close(st[0].double(), mean, rtol=1e-6, atol=1e-6)
    rel = ((got_var - var).abs() / var).max().item()
    assert rel < 2e-3, rel


@pytest.mark.parametrize("mode", ["relu", "res", "ds"])
def test_bn_backward(mode):
    K = _k()
    dtype = torch.bfloat16
    N, H, C = 4, 7, 64
    torch.manual_seed(3)
    y = (torch.randn(N, H, H, C, device=DEV) + 0.3).to(dtype)
    y2 = (torch.randn(N, H, H, C, device=DEV) - 0.2).to(dtype)
    g_in = torch.randn(N, H, H, C, device=DEV).to(dtype)
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    gamma2 = torch.rand(C, device=DEV) + 0.5
    beta2 = torch.randn(C, device=DEV) * 0.1
    # reference with autograd (train-mode batch stats)
    yr = y.float().requires_grad_(True)
    y2r = y2.float().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    g2r = gamma2.clone().requires_grad_(True)
    b2r = beta2.clone().requires_grad_(True)
    _, _, z = _bn_ref(yr, gr, br)
    if mode == "res":
        z = z + y2r
    elif mode == "ds":
        z = z + _bn_ref(y2r, g2r, b2r)[2]
    torch.relu(z).backward(g_in.float())
    # kernel
    ws = K.Workspace(DEV)

    def coeffs(t, ga, be):
        m = t.float().mean((0, 1, 2))
        v = t.float().var((0, 1, 2), unbiased=False)
        inv = 1 / torch.sqrt(v + 1e-5)
        return m, inv, ga * inv, be - m * ga * inv

    m1, i1, s1, h1 = coeffs(y, gamma, beta)
    m2, i2, s2, h2 = coeffs(y2, gamma2, beta2)
    dg = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    dg2 = torch.zeros(C, device=DEV)
    db2 = torch.zeros(C, device=DEV)
    dy = torch.empty_like(y)
    dy2 = torch.empty_like(y)
    dz = torch.empty_like(y)
    if mode == "relu":
        K.bn_bwd(ws, y, m1, i1, gamma, s1, h1, dg, db, dy, g1=g_in)
    elif mode == "res":
        K.bn_bwd(ws, y, m1, i1, gamma, s1, h1, dg, db, dy, g1=g_in, res=y2, dz_buf=dz)
    else:
        K.bn_bwd(ws, y, m1, i1, gamma, s1, h1, dg, db, dy, g1=g_in, y2=y2, mean2=m2, invstd2=i2,
                 gamma2=gamma2, scale2=s2, shift2=h2, dgamma2=dg2, dbeta2=db2, dy2_out=dy2, dz_buf=dz)
    torch.cuda.synchronize()
    assert rel_err(dy, yr.grad) < 2e-2
    assert rel_err(dg, gr.grad) < 1e-2
    assert rel_err(db, br.grad) < 1e-2
    if mode == "res":
        assert rel_err(dz, y2r.grad) < 1e-2
    if mode == "ds":
        assert rel_err(dy2, y2r.grad) < 2e-2
        assert rel_err(dg2, g2r.grad) < 1e-2


def test_stem_pool_and_backward():
    K = _k()
    dtype = torch.bfloat16
    N, H, C = 2, 12, 64
    y = torch.randn(N, H, H, C, device=DEV).to(dtype)
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV) * 0.1
    Ho = (H + 2 - 3) // 2 + 1
    out = torch.empty(N, Ho, Ho, C, device=DEV, dtype=dtype)
    arg = torch.empty(N, Ho, Ho, C, device=DEV, dtype=torch.uint8)
    K.stem_pool(y, sc, sh, out, arg)
    a = torch.relu(y.float() * sc + sh).permute(0, 3, 1, 2).requires_grad_(True)
    ref = F.max_pool2d(a, 3, 2, 1)
    torch.cuda.synchronize()
    assert rel_err(out, ref.permute(0, 2, 3, 1)) < 1e-2
    g = torch.randn_like(ref).to(dtype)
    ref.backward(g.float())
    din = torch.empty_like(y)
    K.maxpool_bwd(g.permute(0, 2, 3, 1).contiguous(), arg, din)
    torch.cuda.synchronize()
    # ties between equal relu outputs (zeros) can route to different windows: compare sums
    torch.testing.assert_close(din.float().sum((1, 2)), a.grad.permute(0, 2, 3, 1).sum((1, 2)),
                               rtol=2e-2, atol=2e-1)


@pytest.mark.parametrize("H", [14, 15])
@pytest.mark.parametrize("with_shortcut", [False, True])
def test_stem_bwd_reduce_matches_unfused(with_shortcut, H):
    """One-pass stem backward (maxpool gather + ReLU mask + BN-backward partials) == maxpool_bwd
    followed by the standalone BN backward, and both == autograd of relu(bn(y)) -> maxpool.
    H = 15: the 2x2-quad work items of the fused kernel hang over the odd bottom/right edge."""
    K = _k()
    dtype = torch.bfloat16
    N, C = 3, 64
    torch.manual_seed(7)
    y = (torch.randn(N, H, H, C, device=DEV) + 0.2).to(dtype)
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    m = y.float().mean((0, 1, 2))
    v = y.float().var((0, 1, 2), unbiased=False)
    inv = 1 / torch.sqrt(v + 1e-5)
    sc, sh = gamma * inv, beta - m * gamma * inv
    Ho = (H + 2 - 3) // 2 + 1
    out = torch.empty(N, Ho, Ho, C, device=DEV, dtype=dtype)
    arg = torch.empty(N, Ho, Ho, C, device=DEV, dtype=torch.uint8)
    K.stem_pool(y, sc, sh, out, arg)
    g = torch.randn(N, Ho, Ho, C, device=DEV).to(dtype)
    g2 = torch.randn(N, Ho, Ho, C, device=DEV).to(dtype) if with_shortcut else None
    ws = K.Workspace(DEV)
    # unfused reference path
    dA = torch.empty_like(y)
    K.maxpool_bwd(g, arg, dA, dout2=g2)
    dy_ref = torch.empty_like(y)
    dg_ref, db_ref = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    K.bn_bwd(ws, y, m, inv, gamma, sc, sh, dg_ref, db_ref, dy_ref, g1=dA)
    # fused
    dz = torch.empty_like(y)
    part, G, nq = K.stem_bwd_reduce(ws, g, arg, y, sc, sh, dz, dout2=g2)
    dy = torch.empty_like(y)
    dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    K.bn_bwd_finish(ws, part, G, nq, y, m, inv, gamma, dg, db, dz, dy)
    torch.cuda.synchronize()
    assert rel_err(dy, dy_ref) < 1e-2
    assert rel_err(dg, dg_ref) < 1e-3 and rel_err(db, db_ref) < 1e-3
    # autograd reference (BN batch statistics + ReLU + max-pool)
    yr = y.float().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    _, _, z = _bn_ref(yr, gr, br)
    ref = F.max_pool2d(torch.relu(z).permute(0, 3, 1, 2), 3, 2, 1)
    gsum = g.float() + (g2.float() if g2 is not None else 0)
    ref.backward(gsum.permute(0, 3, 1, 2))
    assert rel_err(db, br.grad) < 2e-2
    assert rel_err(dg, gr.grad) < 2e-2


def test_tail_pool():
    K = _k()
    dtype = torch.bfloat16
    N, H, C = 3, 7, 256
    y = torch.randn(N, H, H, C, device=DEV).to(dtype)
    r = torch.randn(N, H, H, C, device=DEV).to(dtype)
    sc = torch.rand(C, device=DEV)
    sh = torch.randn(C, device=DEV) * 0.1
    out = torch.empty(N, C, device=DEV, dtype=dtype)
    K.tail_pool(y, sc, sh, out, res=r)
    torch.cuda.synchronize()
    ref = torch.relu(y.float() * sc + sh + r.float()).mean((1, 2))
    assert rel_err(out, ref) < 1e-2


def test_xent_and_topk():
    K = _k()
    B, Cls, ld = 37, 1000, 1024
    logits = torch.randn(B, Cls, device=DEV) * 3
    labels = torch.randint(0, Cls, (B,), device=DEV)
    lr = torch.empty(B, device=DEV)
    loss = torch.empty((), device=DEV)
    dlog = torch.empty(B, ld, device=DEV, dtype=torch.bfloat16)
    K.xent(logits, labels, lr, loss, dlog=dlog, gscale=1.0 / B)
    lref = logits.clone().requires_grad_(True)
    ce = F.cross_entropy(lref, labels)
    ce.backward()
    torch.cuda.synchronize()
    torch.testing.assert_close(loss, ce.detach(), rtol=1e-4, atol=1e-4)
    assert rel_err(dlog[:, :Cls], lref.grad) < 1e-2
    assert dlog[:, Cls:].abs().max().item() == 0
    hits = torch.zeros(2, device=DEV)
    K.topk_hits(logits, labels, hits)
    _, pred = logits.topk(5, -1, True, True)
    h = pred.eq(labels[:, None])
    torch.cuda.synchronize()
    assert hits[0].item() == h[:, :1].sum().item() and hits[1].item() == h.sum().item()


def test_sgd_flat_matches_torch():
    K = _k()
    n = 1000003
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    buf = torch.zeros(n, device=DEV)
    sh = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    pr = torch.nn.Parameter(p.clone())
    opt = torch.optim.SGD([pr], lr=0.1, momentum=0.9, weight_decay=1e-4)
    for it in range(3):
        pr.grad = g.clone()
        opt.step()
        K.sgd_flat(p, g, buf, sh, 0.1, 0.9, 1e-4, initialized=it > 0)
    torch.cuda.synchronize()
    torch.testing.assert_close(p, pr.detach(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(sh.float(), p.to(torch.bfloat16).float())
    # AMP: skipped when found_inf is set, unscaled by the published 1/scale otherwise
    inv = torch.tensor([0.25], device=DEV)
    inf = torch.ones(1, device=DEV)
    before = p.clone()
    K.sgd_flat(p, g, buf, sh, 0.1, 0.9, 1e-4, True, inv_scale=inv, found_inf=inf)
    torch.cuda.synchronize()
    assert torch.equal(before, p)
    pr.grad = g.clone() * 0.25
    opt.step()
    K.sgd_flat(p, g, buf, sh, 0.1, 0.9, 1e-4, True, inv_scale=inv, found_inf=torch.zeros(1, device=DEV))
    torch.cuda.synchronize()
    torch.testing.assert_close(p, pr.detach(), rtol=1e-6, atol=1e-6)


def test_amp_scan_matches_gradscaler_state_machine():
    """amp_scan (non-finite scan + last-workgroup GradScaler update, one launch) against torch's
    own _amp_foreach_non_finite_check_and_unscale_ / _amp_update_scale_ over a sequence of clean
    and overflowing steps (growth interval 3 so growth happens), on a gradient large enough for
    thousands of workgroups -- and with no memset between launches (the kernel resets its own
    arrival counter)."""
    K = _k()
    n = (1 << 22) + 3584
    g = torch.randn(n, device=DEV)
    scale, tracker = torch.tensor([65536.0], device=DEV), torch.zeros(1, dtype=torch.int32, device=DEV)
    s_ref, t_ref = scale.clone(), tracker.clone()
    fi, inv = torch.zeros(1, device=DEV), torch.zeros(1, device=DEV)
    ws = torch.zeros(2, dtype=torch.int32, device=DEV)
    # 1: inf, 2: nan, 3: -inf at the very end, 4: non-finite values in every workgroup
    pattern = [0, 0, 0, 1, 0, 2, 0, 0, 0, 0, 3, 0, 4, 0, 0, 0]
    for step, kind in enumerate(pattern):
        gg = g.clone()
        if kind == 1:
            gg[12345] = float("inf")
        elif kind == 2:
            gg[n // 2] = float("nan")
        elif kind == 3:
            gg[n - 1] = float("-inf")
        elif kind == 4:
            gg[::997] = float("inf")
        fr = torch.zeros(1, device=DEV)
        inv_ref = s_ref.double().reciprocal().float()
        torch._amp_foreach_non_finite_check_and_unscale_([gg.clone()], fr, inv_ref)
        K.amp_scan(gg, fi, inv, scale, tracker, ws, 2.0, 0.5, 3)
        torch.cuda.synchronize()
        assert fi.item() == fr.item(), step
        assert inv.item() == inv_ref.item(), step
        torch._amp_update_scale_(s_ref, t_ref, fr, 2.0, 0.5, 3)
        assert scale.item() == s_ref.item() and tracker.item() == t_ref.item(), (step, scale, s_ref)
        assert ws.tolist() == [0, 0]


def test_synthetic_kernel_matches_torch_generator():
    K = _k()
    from pytorch_distributed_amd.data.synthetic import synthetic_images
    ids = torch.tensor([0, 7, 1281166, 99], device=DEV)
    S = 32
    out = torch.empty(4, S, S, 8, device=DEV, dtype=torch.bfloat16)
    lab = torch.empty(4, dtype=torch.int64, device=DEV)
    keys = torch.empty(4, dtype=torch.int32, device=DEV)
    K.synth_batch(ids, 0, "train", 1000, S, out, lab, keys)
    xr, yr = synthetic_images(ids.cpu(), 0, "train", 1000, S)
    torch.cuda.synchronize()
    assert torch.equal(lab.cpu(), yr)
    torch.testing.assert_close(out[..., :3].float().cpu(), xr.permute(0, 2, 3, 1).to(torch.bfloat16).float(),
                               rtol=1e-2, atol=2e-2)
    assert out[..., 3:].abs().max().item() == 0


@pytest.mark.parametrize("geo", [(2, 8, 64, 128), (8, 16, 64, 64)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("mode", ["relu", "res", "ds", "mask"])
@pytest.mark.parametrize("stride", [1, 2])
def test_dgrad_fused_bn_backward(mode, stride, dtype, geo):
    """dgrad epilogue (mask + BN-backward partial sums) + the one-launch finalize (f64 slabs,
    last-arriver combine: gamma/beta grads and apply coefficients of both branches) == plain dgrad
    followed by the standalone BN-backward reduce / finalize / apply (16-bit and exact-f32
    kernels); the arrival counters are left at zero."""
    K = _k()
    tol = 1e-2 if dtype != torch.float32 else 1e-5
    Nb, H, Cin, Cout = geo
    torch.manual_seed(5)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, 3, 3, stride, 1)
    dy = torch.randn(Nb, g.Ho, g.Wo, Cout, device=DEV).to(dtype)
    w = (torch.randn(Cout, 3, 3, Cin, device=DEV) * 0.05).to(dtype)
    y = torch.randn(Nb, H, H, Cin, device=DEV).to(dtype)
    y2 = torch.randn(Nb, H, H, Cin, device=DEV).to(dtype)
    g2 = torch.randn(Nb, H, H, Cin, device=DEV).to(dtype)
    sc, sh = torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV) * 0.1
    sc2, sh2 = torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV) * 0.1
    mean, inv = torch.randn(Cin, device=DEV) * 0.1, torch.rand(Cin, device=DEV) + 0.5
    mean2, inv2 = torch.randn(Cin, device=DEV) * 0.1, torch.rand(Cin, device=DEV) + 0.5
    gamma, gamma2 = torch.rand(Cin, device=DEV) + 0.5, torch.rand(Cin, device=DEV) + 0.5
    ws = K.Workspace(DEV)
    kw = {}
    if mode in ("res", "mask"):
        kw = dict(res=y2)
    elif mode == "ds":
        kw = dict(y2=y2, scale2=sc2, shift2=sh2)
    use_g2 = mode != "relu"
    # reference: plain dgrad + standalone bn_bwd
    da = torch.empty(Nb, H, H, Cin, device=DEV, dtype=dtype)
    K.conv_dgrad(dy, w, g, da)
    outs_ref = [torch.zeros(Cin, device=DEV) for _ in range(4)]
    dy_ref = torch.empty_like(y)
    dy2_ref = torch.empty_like(y)
    dz_ref = torch.empty_like(y)
    extra = {}
    if mode == "ds":
        extra = dict(mean2=mean2, invstd2=inv2, gamma2=gamma2, dgamma2=outs_ref[2], dbeta2=outs_ref[3],
                     dy2_out=dy2_ref)
    K.bn_bwd(ws, y, mean, inv, gamma, sc, sh, outs_ref[0], outs_ref[1], dy_ref, g1=da,
             g2=g2 if use_g2 else None, dz_buf=dz_ref, **kw, **extra)
    # fused
    G = K.dgrad_slabs(g, Nb)
    if mode == "mask":   # the forward tail's ReLU bitmask replaces the residual read
        mask = torch.empty(y.numel() // 8, dtype=torch.uint8, device=DEV)
        K.bn_apply(y, sc, sh, torch.empty_like(y), res=y2, mask=mask)
        kw = dict(mask=mask)
    outs = [torch.zeros(Cin, device=DEV) for _ in range(4)]
    epi, part, nq = K.bn_epilogue(ws, G, y, sc, sh, g2=g2 if use_g2 else None, **kw)
    dz = torch.empty_like(y)
    K.conv_dgrad(dy, w, g, dz, epi=epi)
    dyf = torch.empty_like(y)
    dy2f = torch.empty_like(y)
    extra = {}
    if mode == "ds":
        extra = dict(y2=y2, mean2=mean2, invstd2=inv2, gamma2=gamma2, dgamma2=outs[2], dbeta2=outs[3],
                     dy2_out=dy2f)
    K.bn_bwd_finish(ws, part, G, nq, y, mean, inv, gamma, outs[0], outs[1], dz, dyf, **extra)
    torch.cuda.synchronize()
    assert int(ws.counters(64).abs().sum().item()) == 0
    if mode != "relu":
        assert rel_err(dz, dz_ref) < tol
    assert rel_err(dyf, dy_ref) < 2 * tol
    for a, b in zip(outs, outs_ref):
        if b.abs().sum() > 0:
            assert rel_err(a, b) < tol
    if mode == "ds":
        assert rel_err(dy2f, dy2_ref) < 2 * tol


@pytest.mark.parametrize("mode", ["exact", "split"])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad_exact_f32(case, mode, monkeypatch):
    """f32 implicit GEMM vs a float64 CPU reference. ``exact`` (MFMA 16x16x4 f32): errors at fp32
    rounding level (no 16-bit operand rounding anywhere). ``split`` (DT_F32S: f32 tensors, bf16
    MFMA on the hi/lo split a_hi*b_hi + a_hi*b_lo + a_lo*b_hi): ~1e-5 relative -- well inside the
    TF32 (10-bit) convolutions of the reference's fp32 runs."""
    K = _k()
    monkeypatch.setattr(K, "_F32_CONV", mode)
    tol = 2e-6 if mode == "exact" else 1e-4
    Nb, H, Cin, Cout, k, s = case
    pad = k // 2
    torch.manual_seed(0)
    x = torch.randn(Nb, Cin, H, H) + 0.1
    w = torch.randn(Cout, Cin, k, k) / math.sqrt(Cin * k * k)
    xd, wd = x.double(), w.double()
    y_ref = F.conv2d(xd, wd, stride=s, padding=pad)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, k, k, s, pad)
    x_nhwc = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    w_ohwi = w.permute(0, 2, 3, 1).contiguous().to(DEV)
    y = torch.empty(Nb, g.Ho, g.Wo, Cout, device=DEV)
    M = Nb * g.Ho * g.Wo
    tile = K.fwd_tile(g, Nb, torch.float32)
    T = K.stats_tiles(M, Cout, tile)
    stats = torch.zeros(T * 3 * Cout, device=DEV)
    K.conv_fwd(x_nhwc, w_ohwi.view(Cout, -1), g, y, stats=stats)
    torch.cuda.synchronize()
    assert rel_err(y.cpu().double(), y_ref.permute(0, 2, 3, 1)) < tol
    st = K.stats_totals(stats, M, Cout, tile[0]).cpu()
    yb = y_ref.permute(0, 2, 3, 1).reshape(-1, Cout)
    torch.testing.assert_close(st[0], yb.sum(0), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(st[1], (yb * yb).sum(0), rtol=1e-4, atol=1e-4)
    dy = torch.randn(y_ref.shape)
    xr = xd.clone().requires_grad_(True)
    wr = wd.clone().requires_grad_(True)
    F.conv2d(xr, wr, stride=s, padding=pad).backward(dy.double())
    dy_nhwc = dy.permute(0, 2, 3, 1).contiguous().to(DEV)
    dx = torch.full((Nb, H, H, Cin), float("nan"), device=DEV)
    K.conv_dgrad(dy_nhwc, w_ohwi, g, dx)
    ws = K.Workspace(DEV)
    dw = torch.zeros(Cout, k, k, Cin, device=DEV)
    K.conv_wgrad(dy_nhwc, x_nhwc, g, dw.view(-1), ws)
    torch.cuda.synchronize()
    assert rel_err(dx.cpu().double(), xr.grad.permute(0, 2, 3, 1)) < tol
    assert rel_err(dw.cpu().double(), wr.grad.permute(0, 2, 3, 1)) < tol


def test_bn_stats_handoff_under_uneven_load():
    """The BN statistics kernel's cross-workgroup hand-off (f64 slabs written write-through, a
    release-ordered arrival counter, the last arriver's acquire) under UNEVEN load: a weight-
    gradient GEMM saturating the CUs on a second stream while the statistics launches run, several
    sizes, repeated in one process; every channel of every launch is checked against float64
    (MI355X_MICROARCH.md: test hand-offs under uneven load, consumer L1-warm)."""
    K = _k()
    dev = torch.device(DEV)
    side = torch.cuda.Stream(dev)
    g = K.ConvGeom(64, 14, 14, 256, 256, 3, 3, 1, 1)
    dy = torch.randn(64, 14, 14, 256, device=dev).to(torch.bfloat16)
    x = torch.randn(64, 14, 14, 256, device=dev).to(torch.bfloat16)
    gw = torch.empty(256 * 9 * 256, device=dev)
    ws_side = K.Workspace(dev)
    ws = K.Workspace(dev)
    bad = []
    for rep in range(6):
        for C, T in ((256, 613), (512, 154), (2048, 77), (64, 9800)):
            torch.manual_seed(rep * 7 + C)
            bm = 128
            M = T * bm - 5
            rows = torch.full((T,), float(bm), dtype=torch.float64)
            rows[-1] = M - (T - 1) * bm
            s1 = torch.randn(T, C, dtype=torch.float64)
            sh = torch.randn(T, C, dtype=torch.float64)
            s2 = torch.rand(T, C, dtype=torch.float64) * 50 + s1 ** 2 / rows[:, None]
            part = torch.stack([s1, s2, sh], 1).float()
            p64 = part.double()
            mean = ((rows[:, None] * p64[:, 2] + p64[:, 0]).sum(0)) / M
            with torch.cuda.stream(side):       # the competing load
                for _ in range(3):
                    K.conv_wgrad(dy, x, g, gw, ws_side)
            gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
            st = torch.zeros(4, C, device=dev)
            bn = K.BnStats(ws, gamma, beta, 1e-5, 0.1, st[0], st[1], st[2], st[3],
                           update_running=False)
            pdev = part.to(dev).contiguous()
            st[0].copy_(pdev[0, 0])              # L1-warm consumer lines with stale values
            K.bn_finalize_partials(pdev, T, C, bm, M, bn)
            torch.cuda.synchronize()
            err = (st[0].double().cpu() - mean).abs().max().item()
            if not err < 1e-4:
                bad.append((rep, C, T, err))
    assert not bad, bad
    assert int(ws.counters(64).abs().sum().item()) == 0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("Cout,Cin", [(256, 64), (512, 128), (2048, 512)])
def test_bn_fold_operands(Cout, Cin, dtype):
    """bn_fold_kernel: Wf = [k1 o W ; W^T diag(k2) W] and b = W^T k3 against fp32 torch on the same
    16-bit weights (G and the k1 rows are rounded to the 16-bit dtype once)."""
    K = _k()
    torch.manual_seed(Cout + Cin)
    w = (torch.randn(Cout, Cin, device=DEV) * 0.05).to(dtype)
    k = torch.randn(3 * Cout, device=DEV)
    wf = torch.empty(Cout + Cin, Cin, device=DEV, dtype=dtype)
    b = torch.empty(Cin, device=DEV)
    K.bn_fold(w, k, wf, b)
    torch.cuda.synchronize()
    wd = w.double()
    k1, k2, k3 = k[:Cout].double(), k[Cout:2 * Cout].double(), k[2 * Cout:].double()
    # the kernel scales the 16-bit W by k2 and rounds that product once before the MFMA
    wk2 = (w.float() * k2.float()[:, None]).to(dtype).double()
    g_ref = wd.t() @ wk2
    assert rel_err(wf[:Cout], (wd * k1[:, None])) < 5e-3
    assert rel_err(wf[Cout:], g_ref) < 5e-3
    assert rel_err(wf[Cout:], wd.t() @ (k2[:, None] * wd)) < 1e-2
    assert rel_err(b, wd.t() @ k3) < 1e-5


@pytest.mark.parametrize("pro", [True, False])
@pytest.mark.parametrize("geo", [(2, 8, 64, 256), (3, 7, 128, 512), (1, 7, 512, 2048)])
def test_conv_dgrad_bnf_matches_applied_dgrad(geo, pro):
    """DGRAD_BNF (the consumer-side tail fold) == apply dy3 = k1*dz + k2*y3 + k3, then the plain 1x1
    data gradient -- with y3 = conv(a2) the conv's own forward, a2 = relu(bn2(y2)) recomputed by the
    prologue (pro) or a materialised input; ragged rows (H = 7); the fused BN-backward epilogue of
    the preceding BN gives the same dz and partial sums."""
    K = _k()
    dtype = torch.bfloat16
    Nb, H, Cin, Cout = geo
    torch.manual_seed(Cin)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, 1, 1, 1, 0)
    w = (torch.randn(Cout, 1, 1, Cin, device=DEV) * 0.05).to(dtype)
    y2 = torch.randn(Nb, H, H, Cin, device=DEV).to(dtype)
    sc2, sh2 = torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV) * 0.1
    if pro:
        xa, xpro = y2, (sc2, sh2)
        a2 = torch.relu(y2.float() * sc2 + sh2).to(dtype)
    else:
        xa, xpro = torch.relu(y2.float()).to(dtype), None
        a2 = xa
    y3 = torch.empty(Nb, H, H, Cout, device=DEV, dtype=dtype)
    K.conv_fwd(a2, w.view(Cout, Cin), g, y3)
    dz = torch.randn(Nb, H, H, Cout, device=DEV).to(dtype)
    k = torch.cat([torch.rand(Cout, device=DEV) + 0.5, torch.randn(Cout, device=DEV) * 0.3,
                   torch.randn(Cout, device=DEV) * 0.2])
    dy3 = (k[:Cout] * dz.float() + k[Cout:2 * Cout] * y3.float() + k[2 * Cout:]).to(dtype)
    ws = K.Workspace(DEV)
    mean, inv = torch.randn(Cin, device=DEV) * 0.1, torch.rand(Cin, device=DEV) + 0.5
    gamma = torch.rand(Cin, device=DEV) + 0.5
    res = {}
    for name in ("ref", "bnf"):
        G = K.dgrad_slabs(g, Nb, dtype=dtype)
        epi, part, nq = K.bn_epilogue(ws, G, y2, sc2, sh2)
        dz2 = torch.empty(Nb, H, H, Cin, device=DEV, dtype=dtype)
        if name == "ref":
            K.conv_dgrad(dy3, w, g, dz2, epi=epi)
        else:
            wf = torch.empty(Cout + Cin, Cin, device=DEV, dtype=dtype)
            b = torch.empty(Cin, device=DEV)
            K.bn_fold(w.view(Cout, Cin), k, wf, b)
            K.conv_dgrad_bnf(dz, wf, g, dz2, xa, b, xa_pro=xpro, epi=epi)
        dg, db = torch.zeros(Cin, device=DEV), torch.zeros(Cin, device=DEV)
        dy2 = torch.empty_like(dz2)
        K.bn_bwd_finish(ws, part, G, nq, y2, mean, inv, gamma, dg, db, dz2, dy2)
        torch.cuda.synchronize()
        res[name] = (dz2.float(), dg.clone(), db.clone())
    # exact-math reference of the data gradient (fp32): dA2 = dY3 . W  (dY3 unrounded)
    dy3f = k[:Cout] * dz.float() + k[Cout:2 * Cout] * y3.float() + k[2 * Cout:]
    da_ref = dy3f.view(-1, Cout) @ w.view(Cout, Cin).float()
    mask = (y2.float() * sc2 + sh2 > 0).view(-1, Cin)
    dz2_ref = (da_ref * mask).view(Nb, H, H, Cin)
    e_bnf, e_ref = rel_err(res["bnf"][0], dz2_ref), rel_err(res["ref"][0], dz2_ref)
    print(f"dz2 vs fp32: fold {e_bnf:.2e}, apply+dgrad {e_ref:.2e}")
    assert e_bnf < 2 * e_ref + 5e-3, (e_bnf, e_ref)
    for a, b in zip(res["bnf"][1:], res["ref"][1:]):
        assert rel_err(a, b) < 1.5e-2


@pytest.mark.parametrize("Cout,Cin,H,tile", [(256, 64, 14, (-128, 128)), (512, 128, 12, (128, 128)),
                                              (1024, 256, 7, (-128, 64)), (2048, 512, 7, (-128, 128))])
def test_conv_wgrad_bna_conv3_tiles(Cout, Cin, H, tile):
    """WGRAD_BNA on the Bottleneck conv3 tiles of the tail fold, with the forward's BN+ReLU
    prologue on the activation operand: against the apply-then-wgrad path."""
    K = _k()
    dtype = torch.bfloat16
    Nb = 4
    torch.manual_seed(Cout)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, 1, 1, 1, 0)
    y2 = torch.randn(Nb, H, H, Cin, device=DEV).to(dtype)
    sc, sh = torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV) * 0.1
    dz = torch.randn(Nb, H, H, Cout, device=DEV).to(dtype)
    y3 = (torch.randn(Nb, H, H, Cout, device=DEV) * 2 + 1).to(dtype)
    kk = torch.randn(3 * Cout, device=DEV)
    ws = K.Workspace(DEV)
    dw_f = torch.zeros(Cout * Cin, device=DEV)
    K.conv_wgrad(dz, y2, g, dw_f, ws, pro=(sc, sh), bna=(y3, kk), tile=tile)
    dy = (kk[:Cout].double() * dz.double() + (kk[Cout:2 * Cout].double() * y3.double()
                                              + kk[2 * Cout:].double()).float().double()).float().to(dtype)
    dw_u = torch.zeros_like(dw_f)
    K.conv_wgrad(dy, y2, g, dw_u, ws, pro=(sc, sh), tile=tile)
    torch.cuda.synchronize()
    assert rel_err(dw_f, dw_u) < 2e-3


@pytest.mark.parametrize("geo", [(2, 8, 64, 256), (2, 14, 256, 512), (1, 14, 512, 1024)])
def test_conv_dgrad_bnf_stride2_shortcut(geo):
    """DGRAD_BNF on a strided 1x1 shortcut conv (the downsample branch of the tail fold): the Gram
    operand is the block input x at the landing pixels, the other parity classes are exact zeros
    (no bias there), against apply-then-plain-dgrad."""
    K = _k()
    dtype = torch.bfloat16
    Nb, H, Cin, Cout = geo
    torch.manual_seed(Cout)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, 1, 1, 2, 0)
    w = (torch.randn(Cout, 1, 1, Cin, device=DEV) * 0.05).to(dtype)
    x = torch.relu(torch.randn(Nb, H, H, Cin, device=DEV)).to(dtype)
    yd = torch.empty(Nb, g.Ho, g.Wo, Cout, device=DEV, dtype=dtype)
    K.conv_fwd(x, w.view(Cout, Cin), g, yd)
    dz = torch.randn(Nb, g.Ho, g.Wo, Cout, device=DEV).to(dtype)
    k = torch.cat([torch.rand(Cout, device=DEV) + 0.5, torch.randn(Cout, device=DEV) * 0.3,
                   torch.randn(Cout, device=DEV) * 0.2])
    dyd = (k[:Cout] * dz.float() + k[Cout:2 * Cout] * yd.float() + k[2 * Cout:]).to(dtype)
    ref = torch.empty(Nb, H, H, Cin, device=DEV, dtype=dtype)
    K.conv_dgrad(dyd, w, g, ref)
    wf = torch.empty(Cout + Cin, Cin, device=DEV, dtype=dtype)
    b = torch.empty(Cin, device=DEV)
    K.bn_fold(w.view(Cout, Cin), k, wf, b)
    out = torch.full((Nb, H, H, Cin), 7.0, device=DEV, dtype=dtype)
    K.conv_dgrad_bnf(dz, wf, g, out, x, b)
    torch.cuda.synchronize()
    exact = ((k[:Cout] * dz.float() + k[Cout:2 * Cout] * yd.float() + k[2 * Cout:]).view(-1, Cout)
             @ w.view(Cout, Cin).float()).view(Nb, g.Ho, g.Wo, Cin)
    land = out[:, ::2, ::2]
    assert out[:, 1::2].abs().max().item() == 0 and out[:, :, 1::2].abs().max().item() == 0
    e_bnf, e_ref = rel_err(land, exact), rel_err(ref[:, ::2, ::2], exact)
    print(f"shortcut dX vs fp32: fold {e_bnf:.2e}, apply+dgrad {e_ref:.2e}")
    assert e_bnf < 2 * e_ref + 5e-3, (e_bnf, e_ref)


@pytest.mark.parametrize("Cout,Cin,H", [(64, 256, 14), (128, 512, 12), (256, 1024, 7), (512, 2048, 7)])
def test_conv_wgrad_bna_conv1_tiles(Cout, Cin, H):
    """WGRAD_BNA on the Bottleneck conv1 shapes of the head fold (M = Cout small, N = Cin = 4 Cout):
    against the apply-then-wgrad path on the plan's own tile."""
    K = _k()
    dtype = torch.bfloat16
    Nb = 4
    torch.manual_seed(Cout)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, 1, 1, 1, 0)
    x = torch.relu(torch.randn(Nb, H, H, Cin, device=DEV)).to(dtype)
    dz = torch.randn(Nb, H, H, Cout, device=DEV).to(dtype)
    y1 = (torch.randn(Nb, H, H, Cout, device=DEV) * 2 + 1).to(dtype)
    kk = torch.randn(3 * Cout, device=DEV)
    ws = K.Workspace(DEV)
    assert K.wgrad_bna_ok(g, Nb, dtype)
    bm, bn, _, _ = K.wgrad_plan(g, Nb, bna=True)
    dw_f = torch.zeros(Cout * Cin, device=DEV)
    K.conv_wgrad(dz, x, g, dw_f, ws, bna=(y1, kk))
    dy = (kk[:Cout].double() * dz.double() + (kk[Cout:2 * Cout].double() * y1.double()
                                              + kk[2 * Cout:].double()).float().double()).float().to(dtype)
    dw_u = torch.zeros_like(dw_f)
    K.conv_wgrad(dy, x, g, dw_u, ws, tile=(bm, bn))
    torch.cuda.synchronize()
    assert rel_err(dw_f, dw_u) < 2e-3


@pytest.mark.parametrize("C,H", [(64, 14), (128, 12), (256, 7), (512, 7)])
def test_conv_wgrad_gram_and_bgemm(C, H):
    """WGRAD_GRAM: Gram(a) = a^T a and the column sums of a = relu(y*sc + sh) (both operands
    staged through the BN+ReLU, rounded to bf16 as the forward's prologue does) against fp64 torch;
    fold_bgemm: W Gram."""
    K = _k()
    dtype = torch.bfloat16
    Nb = 3
    torch.manual_seed(C)
    y = torch.randn(Nb, H, H, C, device=DEV).to(dtype)
    sc, sh = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3
    ws = K.Workspace(DEV)
    ge = torch.empty(C + 1, C, device=DEV)
    K.conv_wgrad_gram(y, sc, sh, ge, ws)
    gram, colsum = ge[:C], ge[C]
    w = (torch.randn(4 * C, C, device=DEV) * 0.05).to(dtype)
    B = torch.empty(4 * C, C, device=DEV)
    K.fold_bgemm(w, gram, B)
    torch.cuda.synchronize()
    a = torch.relu(y.float() * sc + sh).to(dtype).double().view(-1, C)
    assert rel_err(gram, a.t() @ a) < 1e-5
    assert rel_err(colsum, a.sum(0)) < 1e-5
    assert rel_err(B, w.double() @ gram.double()) < 1e-5


@pytest.mark.parametrize("Cout,Cin,H", [(256, 64, 14), (512, 128, 12), (1024, 256, 7)])
def test_conv_wgrad_decomposed_fold(Cout, Cin, H):
    """The decomposed tail-fold weight gradient (plain dz^T a2 + the k-combine in the split-K
    reduce with B = W3 Gram(a2), s = colsum(a2)) against the fp64 dY^T a2 with dY = k1*dz + k2*y3
    + k3 and y3 = conv3(a2) -- and no worse than the WGRAD_BNA path."""
    K = _k()
    dtype = torch.bfloat16
    Nb = 4
    torch.manual_seed(Cout + 1)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, 1, 1, 1, 0)
    y2 = torch.randn(Nb, H, H, Cin, device=DEV).to(dtype)
    sc, sh = torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV) * 0.1
    a2 = torch.relu(y2.float() * sc + sh).to(dtype)
    w = (torch.randn(Cout, Cin, device=DEV) * 0.05).to(dtype)
    y3 = torch.empty(Nb, H, H, Cout, device=DEV, dtype=dtype)
    K.conv_fwd(a2, w, g, y3)
    dz = torch.randn(Nb, H, H, Cout, device=DEV).to(dtype)
    kk = torch.cat([torch.rand(Cout, device=DEV) + 0.5, torch.randn(Cout, device=DEV) * 0.3,
                    torch.randn(Cout, device=DEV) * 0.2])
    ws = K.Workspace(DEV)
    ge = torch.empty(Cin + 1, Cin, device=DEV)
    K.conv_wgrad_gram(y2, sc, sh, ge, ws)
    gram, colsum = ge[:Cin], ge[Cin]
    B = torch.empty(Cout, Cin, device=DEV)
    K.fold_bgemm(w, gram, B)
    dw_dec = torch.zeros(Cout * Cin, device=DEV)
    K.conv_wgrad(dz, y2, g, dw_dec, ws, pro=(sc, sh), combine=(kk, B, colsum))
    dw_bna = torch.zeros(Cout * Cin, device=DEV)
    K.conv_wgrad(dz, y2, g, dw_bna, ws, pro=(sc, sh), bna=(y3, kk))
    torch.cuda.synchronize()
    k1, k2, k3 = (kk[:Cout].double(), kk[Cout:2 * Cout].double(), kk[2 * Cout:].double())
    dy = k1 * dz.double() + k2 * y3.double() + k3
    ref = (dy.view(-1, Cout).t() @ a2.double().view(-1, Cin)).reshape(-1)
    e_dec, e_bna = rel_err(dw_dec, ref), rel_err(dw_bna, ref)
    print(f"dW3 vs fp64: decomposed {e_dec:.2e}, BNA {e_bna:.2e}")
    assert e_dec < e_bna + 2e-3, (e_dec, e_bna)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("geo", [(2, 9, 256, 64), (3, 7, 512, 128), (2, 5, 1024, 256), (1, 7, 2048, 512)])
def test_conv_fwd_tail_matches_apply_then_conv(geo, mode, dtype):
    """FWD_TAIL: conv1 of a block consuming the previous tail a = relu(bn3(y3) + r) (r = the
    residual, mode 1, or bn_d(yd), mode 2) formed while staging, writing a and its ReLU bitmask --
    against bn_apply + the plain conv on the same operands: a, the mask, the conv output and its
    BatchNorm statistics all bit-identical (ragged M: H = 5, 7, 9; 1, 2 and 4 N-tiles)."""
    K = _k()
    Nb, H, Cin, Cout = geo
    torch.manual_seed(Cin + mode)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, 1, 1, 1, 0)
    y3 = torch.randn(Nb, H, H, Cin, device=DEV).to(dtype)
    r = torch.randn(Nb, H, H, Cin, device=DEV).to(dtype)
    sc, sh = torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV) * 0.3
    sc2, sh2 = (torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV) * 0.3) if mode == 2 \
        else (None, None)
    w = (torch.randn(Cout, Cin, device=DEV) / math.sqrt(Cin)).to(dtype)
    M = Nb * H * H
    T = math.ceil(M / 128)
    # reference: the apply pass, then the plain conv on the 128-row tile the fused launch uses
    a_ref = torch.empty_like(y3)
    m_ref = torch.zeros(y3.numel() // 8, dtype=torch.uint8, device=DEV)
    if mode == 1:
        K.bn_apply(y3, sc, sh, a_ref, res=r, mask=m_ref)
    else:
        K.bn_apply(y3, sc, sh, a_ref, y2=r, scale2=sc2, shift2=sh2)
    y_ref = torch.empty(Nb, H, H, Cout, device=DEV, dtype=dtype)
    st_ref = torch.zeros(T * 3 * Cout, device=DEV)
    K.conv_fwd(a_ref, w, g, y_ref, stats=st_ref, tile=(-128, 64 if Cout <= 64 else 128))
    a = torch.full_like(y3, float("nan"))
    m = torch.zeros_like(m_ref)
    y = torch.empty_like(y_ref)
    st = torch.zeros_like(st_ref)
    tail = K.TailIn(r, a, mask=m if mode == 1 else None, sc2=sc2, sh2=sh2)
    K.conv_fwd(y3, w, g, y, stats=st, pro=(sc, sh), tail=tail)
    torch.cuda.synchronize()
    assert torch.equal(a, a_ref)
    if mode == 1:
        assert torch.equal(m, m_ref)
    assert torch.equal(y, y_ref)
    assert torch.equal(st, st_ref)


@pytest.mark.parametrize("Nb,H", [(2, 11), (3, 20), (2, 56)])
def test_stem_wgrad_decomposed_matches_bna(Nb, H):
    """The decomposed stem weight gradient (models/native.py stem_split): B = y^T X by the plain
    weight-gradient GEMM, s = per-tap column sums of X (stem_tap_colsum), then plain dz^T X with
    k1 * . + k2 * B + k3 * s in the split-K reduce -- against the fp32 weight gradient of
    dY = k1 dz + k2 y + k3 and against WGRAD_BNA (which rounds dY to bf16: the decomposed form
    is at least as close)."""
    K = _k()
    dtype = torch.bfloat16
    torch.manual_seed(Nb * H + 1)
    g = K.stem_s2d_geom(Nb, 2 * H)
    x = torch.randn(Nb, H, H, 16, device=DEV).to(dtype)
    dz = torch.randn(Nb, H, H, 64, device=DEV).to(dtype)
    y = (torch.randn(Nb, H, H, 64, device=DEV) * 2 + 1).to(dtype)
    kk = torch.randn(3 * 64, device=DEV)
    dy = (kk[:64].double() * dz.double() + kk[64:128].double() * y.double() + kk[128:].double())
    dyp = torch.zeros(Nb, 64, H + 1, H + 1, device=DEV, dtype=torch.float64)
    dyp[:, :, :H, :H] = dy.permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (64, 16, 4, 4), dyp, padding=2)
    ref = ref.permute(0, 2, 3, 1).reshape(-1).float()
    ws = K.Workspace(torch.device(DEV))
    B = torch.empty(64 * 256, device=DEV)
    K.conv_wgrad(y, x, g, B, ws)
    s = K.stem_tap_colsum(x, g)
    dec = torch.full((64 * 256,), float("nan"), device=DEV)
    K.conv_wgrad(dz, x, g, dec, ws, combine=(kk, B, s))
    bna = torch.zeros(64 * 256, device=DEV)
    K.conv_wgrad(dz, x, g, bna, ws, bna=(y, kk))
    torch.cuda.synchronize()
    e_dec, e_bna = rel_err(dec, ref), rel_err(bna, ref)
    assert e_dec < e_bna + 1e-4, (e_dec, e_bna)
    assert e_dec < 1e-3, e_dec


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("Nb,H", [(2, 11), (3, 20), (2, 112)])
def test_wgrad_stem_tap_matches_fp32_and_bna(Nb, H, dtype):
    """csrc/wgrad_tap.hip wgrad_stem_tap_kernel: the stem's weight gradient (4x4 / stride 1 / pad
    2 on the 16-channel space-to-depth image, output cropped to H x H) with dY = k1*dz + k2*y + k3
    formed in LDS, all 16 taps per block, against the fp32 reference of the same dY and against the
    implicit-GEMM WGRAD_BNA tile; several split counts (ragged last split); deterministic."""
    K = _k()
    torch.manual_seed(Nb * H)
    g = K.stem_s2d_geom(Nb, 2 * H)
    if not K.stem_wgrad_tap_ok(g, dtype, force=True):
        pytest.skip("stem tap kernel not built")
    x = torch.randn(Nb, H, H, 16, device=DEV).to(dtype)
    dz = torch.randn(Nb, H, H, 64, device=DEV).to(dtype)
    y = (torch.randn(Nb, H, H, 64, device=DEV) * 2 + 1).to(dtype)
    kk = torch.randn(3 * 64, device=DEV)
    dy = (kk[:64].double() * dz.double() + (kk[64:128].double() * y.double()
                                            + kk[128:].double()).float().double()).float().to(dtype)
    dyp = torch.zeros(Nb, 64, H + 1, H + 1, device=DEV)
    dyp[:, :, :H, :H] = dy.float().permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 16, 4, 4), dyp, padding=2)
    ref = ref.permute(0, 2, 3, 1).contiguous()          # OHWI
    ws = K.Workspace(torch.device(DEV))
    gen = torch.zeros(64 * 256, device=DEV)
    K.conv_wgrad(dz, x, g, gen, ws, bna=(y, kk), tile=(-64, 256))   # the generic WGRAD_BNA tile
    outs = []
    for blocks in (5, 64, 512):
        gw = torch.full((64 * 256,), float("nan"), device=DEV)
        K.conv_wgrad_stem_tap(dz, y, kk, x, g, gw, ws, blocks=blocks)
        outs.append(gw.clone())
    again = torch.full_like(outs[-1], float("nan"))
    K.conv_wgrad_stem_tap(dz, y, kk, x, g, again, ws, blocks=512)
    torch.cuda.synchronize()
    e_gen = rel_err(gen.view_as(ref), ref)
    for o in outs:
        e = rel_err(o.view_as(ref), ref)
        assert e < 2 * e_gen + 1e-5, (e, e_gen)
    assert torch.equal(again, outs[-1])   # deterministic run to run


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("geo", [(2, 56, 64, 64, False), (2, 56, 64, 64, True), (3, 28, 128, 128, False),
                                 (2, 28, 64, 128, True), (3, 14, 256, 256, False), (5, 7, 128, 64, True)])
def test_wgrad_tap_matches_fp32_and_generic(geo, dtype):
    """csrc/wgrad_tap.hip: the 3x3 stride-1 weight gradient with all nine taps per block (padded
    pixel rows, X in an LDS ring, BN+ReLU prologue applied in LDS) against the fp32 reference on the
    same 16-bit operands and against the generic implicit-GEMM weight gradient; bitwise
    deterministic run to run; several split counts (last split ragged), Cin != Cout."""
    K = _k()
    Nb, H, Cin, Cout, pro = geo
    torch.manual_seed(H + Cin)
    g = K.ConvGeom(Nb, H, H, Cin, Cout, 3, 3, 1, 1)
    x = (torch.randn(Nb, H, H, Cin, device=DEV) + 0.2).to(dtype)
    dy = (torch.randn(Nb, H, H, Cout, device=DEV) * 0.1).to(dtype)
    sc = torch.rand(Cin, device=DEV) + 0.5 if pro else None
    sh = torch.randn(Cin, device=DEV) * 0.3 if pro else None
    xa = torch.relu(x.float() * sc + sh).to(dtype).float() if pro else x.float()
    ref = torch.nn.grad.conv2d_weight(xa.permute(0, 3, 1, 2), (Cout, Cin, 3, 3),
                                      dy.float().permute(0, 3, 1, 2), padding=1)
    ref = ref.permute(0, 2, 3, 1).contiguous()          # OHWI
    ws = K.Workspace(torch.device(DEV))
    p = (sc, sh) if pro else None
    outs = []
    for blocks in (7, 64, 256):
        gw = torch.full((Cout * 9 * Cin,), float("nan"), device=DEV)
        kb, splits = K.wgrad_tap_plan(g, Nb, blocks)
        slab = ws.get("wgrad_slab", splits * Cout * 9 * Cin)
        L = K.ext.lib()
        K.check(L.pda_wgrad_tap(K.ptr(dy), K.ptr(x), K.ptr(slab), K.ptr(sc), K.ptr(sh), Nb, H, H,
                                Cin, Cout, kb, splits, K.ext.dt_of(dy), K.stream(torch.device(DEV))), "tap")
        K.check(L.pda_wgrad_reduce(K.ptr(slab), K.ptr(gw), splits, Cout, 9 * Cin, int(math.log2(Cin)),
                                   Cin, 9 * Cin, 1.0, 0, None, None, None, K.stream(torch.device(DEV))),
                "reduce")
        outs.append(gw.clone())
    gen = torch.zeros(Cout * 9 * Cin, device=DEV)
    K.conv_wgrad(dy, x, g, gen, ws, pro=p, tile=(-128, 128))   # the generic kernel
    again = torch.full_like(outs[-1], float("nan"))
    K.conv_wgrad_tap(dy, x, g, again, ws, pro=p)
    torch.cuda.synchronize()
    e_gen = rel_err(gen.view_as(ref), ref)
    for o in outs:
        e = rel_err(o.view_as(ref), ref)
        assert e < 2 * e_gen + 1e-5, (e, e_gen)
    k2 = K.conv_wgrad_tap(dy, x, g, torch.empty_like(again), ws, pro=p)
    torch.cuda.synchronize()
    assert torch.equal(again, k2)


def test_wgrad_reduce_batch_matches_single_reduces():
    """native_ops.ReduceBatch: several weight gradients (1x1, 3x3 tap-reuse, the decomposed-fold
    combine, accumulate, the stem's padded-channel remap) with their split-K reductions queued and run
    in ONE launch, against the same weight gradients reduced one launch each (equal to f32 rounding:
    the batched kernel sums the splits in its own fixed order) and bitwise run to run."""
    K = _k()
    dev = torch.device(DEV)
    dtype = torch.bfloat16
    torch.manual_seed(5)
    cases = [K.ConvGeom(4, 14, 14, 256, 64, 1, 1, 1, 0), K.ConvGeom(2, 28, 28, 128, 128, 3, 3, 1, 1),
             K.ConvGeom(3, 7, 7, 512, 512, 3, 3, 1, 1), K.ConvGeom(2, 56, 56, 64, 64, 3, 3, 1, 1)]
    ops = []
    for g in cases:
        x = torch.randn(g.Nb, g.H, g.W, g.Cin, device=dev).to(dtype)
        dy = (torch.randn(g.Nb, g.Ho, g.Wo, g.Cout, device=dev) * 0.1).to(dtype)
        ops.append((g, dy, x))
    g1 = cases[0]
    k = torch.randn(3 * g1.Cout, device=dev)
    cB = torch.randn(g1.Cout, g1.Cin, device=dev)
    cs = torch.randn(g1.Cin, device=dev)

    def run(batched):
        ws = K.Workspace(dev)
        if batched:
            ws.reduce_batch = K.ReduceBatch(ws)
        outs = []
        for n, (g, dy, x) in enumerate(ops):
            o = torch.full((g.Cout * g.R * g.S * g.Cin,), 0.5, device=dev)
            K.conv_wgrad(dy, x, g, o, ws, scale=0.25, accumulate=n == 1,
                         combine=(k, cB, cs) if n == 0 else None)
            outs.append(o)
        if batched:
            assert len(ws.reduce_batch.items) == len(ops)
            ws.reduce_batch.flush()
        torch.cuda.synchronize()
        return outs
    single, batch, again = run(False), run(True), run(True)
    for a, b, c in zip(single, batch, again):
        assert rel_err(b, a) < 1e-6, rel_err(b, a)
        assert torch.equal(b, c)
