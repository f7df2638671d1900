"""The fp32 default's precision (MX_F32_CONV=split: f32 tensors, convolutions on the bf16 MFMA as a
hi/lo three-term split) pinned against TF32, the precision of the reference's fp32 runs.

The reference's fp32 scripts run without autocast on A100, where cuDNN convolutions use TF32 by
default (``/root/reference/resnet_single_gpu.py:27-31``): operands rounded to a 10-bit mantissa,
products and sums in f32. For every convolution of ResNet-50 (the 23 shapes of SURVEY §2.7 and the
space-to-depth stem) and every pass (forward, data gradient, weight gradient), the native split
path's error against float64 must be at or below the error of TF32 operand rounding on the same
inputs (emulated: TF32-rounded operands, the convolution in float64 -- which leaves out TF32's f32
accumulation error, so the bar is stricter than TF32 itself). Batch 1 (2 for the 7x7 layers): the
per-element error of a conv does not depend on the batch size."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (name, H, Cin, Cout, k, stride)
SHAPES = [
    ("C1", 56, 64, 64, 1, 1), ("C2", 56, 64, 64, 3, 1), ("C3", 56, 64, 256, 1, 1),
    ("C4", 56, 256, 64, 1, 1), ("C5", 56, 256, 128, 1, 1), ("C6", 56, 128, 128, 3, 2),
    ("C7", 28, 128, 512, 1, 1), ("C8", 56, 256, 512, 1, 2), ("C9", 28, 512, 128, 1, 1),
    ("C10", 28, 128, 128, 3, 1), ("C11", 28, 512, 256, 1, 1), ("C12", 28, 256, 256, 3, 2),
    ("C13", 14, 256, 1024, 1, 1), ("C14", 28, 512, 1024, 1, 2), ("C15", 14, 1024, 256, 1, 1),
    ("C16", 14, 256, 256, 3, 1), ("C17", 14, 1024, 512, 1, 1), ("C18", 14, 512, 512, 3, 2),
    ("C19", 7, 512, 2048, 1, 1), ("C20", 14, 1024, 2048, 1, 2), ("C21", 7, 2048, 512, 1, 1),
    ("C22", 7, 512, 512, 3, 1),
]


def _k():
    from pytorch_distributed_amd.ops import ext
    ext.load(required=True)
    from pytorch_distributed_amd.ops import native_ops as K
    return K


def tf32(t: torch.Tensor) -> torch.Tensor:
    """Round f32 values to TF32 (10-bit mantissa, round to nearest, ties away from zero)."""
    i = t.float().contiguous().view(torch.int32)
    return ((i + 0x1000) & ~0x1FFF).view(torch.float32)


def rel(a: torch.Tensor, ref: torch.Tensor) -> float:
    a, ref = a.double(), ref.double()
    return ((a - ref).norm() / ref.norm()).item()


def _case(K, name, H, Cin, Cout, k, s):
    Nb = 2 if H == 7 else 1
    pad = k // 2
    torch.manual_seed(int(name[1:]))
    x = torch.randn(Nb, Cin, H, H) * 0.5 + 0.2              # asymmetric activations (post-ReLU-like)
    w = torch.randn(Cout, Cin, k, k) * math.sqrt(2.0 / (Cout * k * k))   # kaiming fan_out
    g = K.ConvGeom(Nb, H, H, Cin, Cout, k, k, s, pad)
    dy = torch.randn(Nb, Cout, g.Ho, g.Wo) * 1e-3
    return Nb, pad, x, w, dy, g


def _ref_grads(x, w, dy, s, pad):
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    y = F.conv2d(xr, wr, stride=s, padding=pad)
    y.backward(dy.double())
    return y.detach(), xr.grad, wr.grad


def _native(K, x, w, dy, g):
    """Forward, data gradient and weight gradient on the native fp32 default (split)."""
    Nb, Cout = x.shape[0], w.shape[0]
    x_nhwc = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    w_ohwi = w.permute(0, 2, 3, 1).contiguous().to(DEV)
    dy_nhwc = dy.permute(0, 2, 3, 1).contiguous().to(DEV)
    y = torch.empty(Nb, g.Ho, g.Wo, Cout, device=DEV)
    K.conv_fwd(x_nhwc, w_ohwi.view(Cout, -1), g, y)
    dx = torch.full((Nb, g.H, g.W, g.Cin), float("nan"), device=DEV)
    K.conv_dgrad(dy_nhwc, w_ohwi, g, dx)
    dw = torch.zeros(Cout, g.R, g.S, g.Cin, device=DEV)
    K.conv_wgrad(dy_nhwc, x_nhwc, g, dw.view(-1), K.Workspace(torch.device(DEV)))
    torch.cuda.synchronize()
    return (y.cpu().permute(0, 3, 1, 2), dx.cpu().permute(0, 3, 1, 2),
            dw.cpu().permute(0, 3, 1, 2))


@pytest.mark.parametrize("shape", SHAPES, ids=[s[0] for s in SHAPES])
def test_split_f32_conv_at_or_below_tf32_error(shape):
    K = _k()
    assert K._F32_CONV == "split", "the fp32 default must be the split convolutions"
    assert K._kdt(torch.empty(0)) == 3
    name, H, Cin, Cout, k, s = shape
    Nb, pad, x, w, dy, g = _case(K, *shape)
    y64, dx64, dw64 = _ref_grads(x, w, dy, s, pad)
    # TF32 operand rounding, the convolution itself in float64
    yt, dxt, dwt = _ref_grads(tf32(x), tf32(w), tf32(dy), s, pad)
    yn, dxn, dwn = _native(K, x, w, dy, g)
    errs = {"fwd": (rel(yn, y64), rel(yt, y64)), "dgrad": (rel(dxn, dx64), rel(dxt, dx64)),
            "wgrad": (rel(dwn, dw64), rel(dwt, dw64))}
    print(name, {p: f"split {e:.2e} tf32 {t:.2e}" for p, (e, t) in errs.items()})
    for p, (e, t) in errs.items():
        assert e <= t, f"{name} {p}: split f32 error {e:.3e} above TF32's {t:.3e}"


def test_split_f32_stem_at_or_below_tf32_error():
    """The stem as the engine runs it in fp32: the 4x4/1 conv on the space-to-depth image (16
    channels, the 7x7/2 weights scattered into the 4x4x16 form), forward and weight gradient."""
    K = _k()
    g = K.stem_s2d_geom(1, 224)
    torch.manual_seed(3)
    x = torch.randn(1, g.Cin, g.H, g.W) * 0.5
    w = torch.randn(g.Cout, g.Cin, 4, 4) * math.sqrt(2.0 / (64 * 49))
    dy = torch.randn(1, g.Cout, g.Ho, g.Wo) * 1e-3

    def ref(x, w, dy):
        xr = F.pad(x.double(), (2, 1, 2, 1)).requires_grad_(True)
        wr = w.double().requires_grad_(True)
        y = F.conv2d(xr, wr)
        y.backward(dy.double())
        return y.detach(), wr.grad
    y64, dw64 = ref(x, w, dy)
    yt, dwt = ref(tf32(x), tf32(w), tf32(dy))
    x_nhwc = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    w_ohwi = w.permute(0, 2, 3, 1).contiguous().to(DEV)
    y = torch.empty(1, g.Ho, g.Wo, g.Cout, device=DEV)
    K.conv_fwd(x_nhwc, w_ohwi.view(g.Cout, -1), g, y)
    dw = torch.zeros(g.Cout, 4, 4, g.Cin, device=DEV)
    K.conv_wgrad(dy.permute(0, 2, 3, 1).contiguous().to(DEV), x_nhwc, g, dw.view(-1),
                 K.Workspace(torch.device(DEV)))
    torch.cuda.synchronize()
    e_f, t_f = rel(y.cpu().permute(0, 3, 1, 2), y64), rel(yt, y64)
    e_w, t_w = rel(dw.cpu().permute(0, 3, 1, 2), dw64), rel(dwt, dw64)
    print(f"stem fwd split {e_f:.2e} tf32 {t_f:.2e}; wgrad split {e_w:.2e} tf32 {t_w:.2e}")
    assert e_f <= t_f and e_w <= t_w
