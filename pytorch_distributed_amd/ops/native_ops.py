"""Op-level Python API over the gfx950 kernels (torch tensors in, torch tensors out).

Layout conventions: activations are NHWC 16-bit (bf16 or f16) tensors of shape
``[N, H, W, C]``; conv weights are 16-bit OHWI ``[Cout, R, S, Cin]`` (the stem
uses a packed ``[64, 448]`` image, see :func:`pack_stem`); statistics, BN
parameters, gradients and the optimizer state are f32.

These functions are what the native ResNet engine
(:mod:`pytorch_distributed_amd.models.native`) schedules, and what the GPU
numerics tests compare against plain PyTorch fp32 references.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch

from . import ext
from .ext import ConvDesc, BwdArgs, check, dt_of, ptr, stream

__all__ = [
    "ConvGeom", "conv_fwd", "conv_dgrad", "conv_wgrad", "pick_tile", "fwd_tile", "wgrad_plan",
    "BnStats", "stats_totals", "bn_finalize_tot", "bn_finalize_partials", "bn_eval_coeffs",
    "bn_apply", "stem_pool", "maxpool_bwd", "tail_pool", "bn_epilogue", "bn_bwd_finish",
    "bn_bwd", "xent", "topk_hits", "col_sum", "sgd_flat", "cast_flat", "amp_scan",
    "pack_stem", "synth_batch", "nchw_to_nhwc8", "Workspace",
]


@dataclass(frozen=True)
class ConvGeom:
    Nb: int
    H: int
    W: int
    Cin: int     # channels of the stored input (stem: 8, padded from 3)
    Cout: int
    R: int
    S: int
    stride: int
    pad: int
    ho: Optional[int] = None   # explicit output size (asymmetric-padding forms, e.g. the s2d stem)
    wo: Optional[int] = None

    @property
    def Ho(self) -> int:
        return self.ho if self.ho is not None else (self.H + 2 * self.pad - self.R) // self.stride + 1

    @property
    def Wo(self) -> int:
        return self.wo if self.wo is not None else (self.W + 2 * self.pad - self.S) // self.stride + 1

    def desc(self, Nb: Optional[int] = None) -> ConvDesc:
        return ConvDesc(self.Nb if Nb is None else Nb, self.H, self.W, self.Cin, self.Cout, self.R,
                        self.S, self.stride, self.pad, self.Ho, self.Wo)

    def with_batch(self, Nb: int) -> "ConvGeom":
        return ConvGeom(Nb, self.H, self.W, self.Cin, self.Cout, self.R, self.S, self.stride, self.pad,
                        self.ho, self.wo)


class ReduceBatch:
    """Split-K reductions queued instead of launched one by one (:func:`conv_wgrad` on a
    :class:`Workspace` whose ``reduce_batch`` is set): each queued weight gradient gets a slab of its
    own, and :meth:`flush` reduces all of them in ONE launch (csrc/conv_gemm.hip
    wgrad_reduce_batch_kernel: the same fixed-order sums, deterministic). The owner flushes on the
    stream the weight gradients ran on, before anything reads the gradients."""

    MAX = 24

    def __init__(self, ws: "Workspace") -> None:
        self.ws = ws
        self.items = []
        self._keep = []

    def slab(self, numel: int) -> torch.Tensor:
        if len(self.items) >= self.MAX:
            self.flush()
        return self.ws.get(f"wgrad_slab_b{len(self.items)}", numel)

    def add(self, slab, grad, splits, M, N, cin_log2, cin_real, pitch, scale, accumulate,
            ck=None, cB=None, cs=None) -> None:
        self.items.append(ext.RedDescC(ptr(slab), ptr(grad), ptr(ck), ptr(cB), ptr(cs), splits, M, N,
                                       cin_log2, cin_real, pitch, int(accumulate), float(scale)))
        self._keep.extend(t for t in (ck, cB, cs) if t is not None)

    def flush(self) -> None:
        if not self.items:
            return
        arr = (ext.RedDescC * len(self.items))(*self.items)
        check(ext.lib().pda_wgrad_reduce_batch(arr, len(self.items), stream(self.ws.device)),
              "wgrad_reduce_batch")
        self.items = []
        self._keep = []


class Workspace:
    """Grow-only scratch buffers (split-K slabs, BN partials) reused by every layer on a stream.

    ``sync_comm``: when set (SyncBatchNorm, :func:`~pytorch_distributed_amd.parallel.ddp.
    convert_sync_batchnorm`), every BatchNorm finalize of this workspace first all-reduces its
    per-channel sums over the communicator, so statistics and their gradients are global."""

    def __init__(self, device) -> None:
        self.device = device
        self._bufs = {}
        self._retired = []   # outgrown buffers stay allocated: a captured HIP graph may use them
        self.sync_comm = None
        self.reduce_batch: Optional[ReduceBatch] = None   # set: conv_wgrad queues its reduce

    def get(self, name: str, numel: int, dtype=torch.float32) -> torch.Tensor:
        b = self._bufs.get(name)
        if b is None or b.numel() < numel or b.dtype != dtype:
            if b is not None:
                self._retired.append(b)
            b = torch.empty(max(numel, 1), dtype=dtype, device=self.device)
            self._bufs[name] = b
        return b[:numel]

    def counters(self, numel: int, name: str = "_counters") -> torch.Tensor:
        """int32 arrival counters of the one-launch reduction kernels: zero when allocated, and
        every kernel that uses them leaves them zero again (its last arrivers reset them). One
        ``name`` per kernel family that may run concurrently with another on the stream."""
        b = self._bufs.get(name)
        if b is None or b.numel() < numel:
            if b is not None:
                self._retired.append(b)
            b = torch.zeros(max(numel, 64), dtype=torch.int32, device=self.device)
            self._bufs[name] = b
        return b[:numel]


_NUM_CU = 256
_WGRAD_TARGET = 2 * _NUM_CU   # default split-K block target of the weight gradients
# every weight-gradient block target x 0.7 in the step: the targets above were tuned per kernel in
# isolation, but a weight gradient shares the device with the main-stream chain, and fewer,
# longer split-K blocks leave it more CUs (bench.py, 5 alternating rounds on one box: x1.0 28.20,
# x0.85 28.15, x0.7 28.04, x0.6 28.11, x0.4 28.24, x1.5 28.34 ms/step; profiles/ab_r3_dma.md)
_WGRAD_SCALE = float(os.environ.get("PDA_WGRAD_SCALE", "0.7"))


# f32 convolutions: "split" (default) = f32 tensors with the products on the bf16 MFMA as a
# three-term hi/lo split (DT_F32S, ~16 significant bits per product: every ResNet-50 conv pass at
# or below the error of TF32 convolutions -- the reference's fp32 runs on A100 -- against float64,
# tests/test_f32_precision_gpu.py; 1.6x the exact path); "exact" = MFMA 16x16x4 f32 (DT_F32, f32
# rounding only; csrc/common.h DType)
_F32_CONV = os.environ.get("PDA_F32_CONV", os.environ.get("MX_F32_CONV", "split"))
if _F32_CONV not in ("exact", "split"):
    raise ValueError(f"MX_F32_CONV / PDA_F32_CONV must be exact|split, got {_F32_CONV!r}")
_SPLIT_BN = 128      # widest N tile of the split kernels
_STEM_G = 4096       # block cap of the one-pass stem backward (profiles/ab_r2_inlaunch_bn.md)
# downsample-tail BN backward: both branches' apply in one pass over dz (False: two launches, kept
# for tests/test_native_model_gpu.py's bitwise parity test of the two forms)
_BWD_APPLY2 = True


def _kdt(t: torch.Tensor) -> int:
    """Kernel dtype code of a conv launch on tensor ``t`` (see _F32_CONV)."""
    d = dt_of(t)
    return 3 if d == 0 and _F32_CONV == "split" else d


def tile_rows(bm: int) -> int:
    """M rows of a tile code: -bm = single-stage register-staged, bm > 1000 = the LDS-DMA 8-wave
    variant of (bm - 1000) rows, bm > 2000 = its tap-reuse form for 3x3 stride-1 fwd / dgrad
    (csrc/conv_gemm.hip dispatch)."""
    return bm - 2000 if bm > 2000 else bm - 1000 if bm > 1000 else abs(bm)


def _ktile(bm: int, bn: int, kdt: int, pro: bool = False) -> Tuple[int, int]:
    """The tile a launch actually uses. The LDS-DMA tiles (bm > 1000) are 16-bit only and cannot
    apply an operand prologue (the bytes never pass through registers): those launches fall back
    to the register-staged 128-row tile. The split-f32 kernels stage hi + lo tiles: single-stage
    tiles of at most 128 x 128."""
    if bm > 1000 and (kdt not in (1, 2) or pro):   # (the HALO tiles too)
        bm, bn = -128, min(bn, 128)
    if kdt != 3:
        return bm, bn
    return -min(abs(bm), 128), min(bn, _SPLIT_BN)


def pick_tile(M: int, N: int, K: Optional[int] = None, dma: bool = False) -> Tuple[int, int]:
    """(bm, bn) for an implicit GEMM; a negative bm selects the single-LDS-buffer variant: half the
    LDS admits a third resident block per CU, which hides the global-load latency better than
    double buffering does at two blocks per CU (measured on all 23 ResNet-50 shapes). ``dma``
    (forward launches): the LDS-DMA 128x256 tile where it measured faster -- deep K (>= 1024) and
    >= 256 output channels with enough tiles for every CU (profiles/convbench_r3_dma.txt: C12 C16
    C17 C18 C20 C22, 4-9 %); the launch falls back to the 128-row register tile when the operand
    needs the BN prologue or is not 16-bit (:func:`_ktile`)."""
    if (dma and _DMA and K is not None and K >= 1024 and N >= 256 and N % 256 == 0
            and math.ceil(M / 128) * (N // 256) >= _NUM_CU):
        return 1128, 256
    bn = 64 if N <= 64 else 128
    bm = 128
    if math.ceil(M / 128) * math.ceil(N / bn) < 2 * _NUM_CU:
        bm = 64
    if bm == 128:
        bm = -128     # single-stage: measured faster on every ResNet-50 shape (tools/conv_bench.py)
    return bm, bn


# ------------------------------------------------------------------ conv
class BnStats:
    """BatchNorm (training) statistics of a conv forward: the conv epilogue writes per-M-tile
    shifted partial sums, which ONE follow-up launch (:func:`bn_finalize_partials`) combines in f64
    and finalizes into mean / invstd / scale / shift and the running statistics. (Finalizing inside
    the conv launch itself measured slower: the finalize code costs the conv epilogue ~2% even when
    idle -- profiles/ab_r2_inlaunch_bn.md.) With SyncBatchNorm (``ws.sync_comm``) the launch stops
    at f64 totals, all-reduced before a small finalize kernel."""

    def __init__(self, ws: "Workspace", gamma, beta, eps: float, momentum: float, mean, invstd,
                 scale, shift, rmean=None, rvar=None, nbt=None, update_running: bool = True):
        self.ws, self.gamma, self.beta = ws, gamma, beta
        self.eps, self.momentum = float(eps), float(momentum)
        self.mean, self.invstd, self.scale, self.shift = mean, invstd, scale, shift
        self.rmean, self.rvar, self.nbt, self.update = rmean, rvar, nbt, update_running


def fwd_tile(g: ConvGeom, Nb: int, dtype: torch.dtype, pro: bool = False,
             Kpad: Optional[int] = None) -> Tuple[int, int]:
    """Default tile of a forward conv. The LDS-DMA tiles take 16-bit operands without the BN
    prologue (their bytes never pass through registers): tap reuse (HALO) on the 3x3 stride-1
    layers with >= 128 output channels (C10 118 -> 105 us, C16 114 -> 98, C22 127 -> 109); other
    launches keep the register-staged choice."""
    dma = _kdt(torch.empty(0, dtype=dtype)) in (1, 2) and not pro and g.Cin >= 64
    if dma and _DMA and _halo_geom(g) and g.Cout >= 128:
        return 2256, 128
    M = Nb * g.Ho * g.Wo
    # (the 128x256 LDS-DMA tile wins 4-9 % per kernel on the deep-K layers but loses in the step:
    # 28.65 -> 28.52 ms/step without it, profiles/ab_r3_dma.md section 12; explicit tile only)
    return pick_tile(M, g.Cout, Kpad if Kpad is not None else g.R * g.S * g.Cin)


def conv_fwd(x: torch.Tensor, w: torch.Tensor, g: ConvGeom, out: torch.Tensor,
             stats: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None,
             relu: bool = False, tile: Optional[Tuple[int, int]] = None,
             pro: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
             bn: Optional[BnStats] = None, before_finalize=None,
             tail: Optional["TailIn"] = None) -> torch.Tensor:
    """out[M, Cout] (16-bit or f32) = conv(x, w). w: [Cout, Kpad] 16-bit, Kpad = w.shape[1].
    stats (f32, >= ceil(M/bm)*3*Cout) receives per-M-tile shifted partials (sum(y-s),
    sum((y-s)^2), s) -- see :func:`stats_totals`; ``bn`` (:class:`BnStats`) also finalizes the
    BatchNorm from them. pro = (scale, shift): x is a PRE-BatchNorm tensor and the conv consumes
    relu(x*scale+shift). ``tail`` (:class:`TailIn`, 1x1 stride-1 convs, see :func:`tail_fuse_ok`):
    x is the previous block's pre-BN tail y3 and the conv consumes a = relu(bn3(y3) + r), writing a
    (and its ReLU bitmask) on the way -- the tail's BN-apply pass folded into its consumer."""
    if tail is not None:
        return _conv_fwd_tail(x, w, g, out, pro, tail, stats, bn, before_finalize)
    Nb = x.shape[0]
    M = Nb * g.Ho * g.Wo
    Kpad = w.shape[-1] if w.dim() == 2 else w[0].numel()
    dense = (tile is None and bias is None and not relu and out.dtype == x.dtype
             and x.is_contiguous() and out.is_contiguous() and w.is_contiguous()
             and x.numel() == Nb * g.H * g.W * g.Cin and out.numel() == M * g.Cout)
    # (the stem kernel writes one statistics partial per output ROW, not per fwd_tile M-tile: a
    # caller-sized ``stats`` buffer without ``bn`` keeps the generic tile's layout)
    if dense and pro is None and Kpad == 256 and (stats is None or bn is not None) \
            and stem_fwd_ok(g, x.dtype):
        return stem_fwd(x, w, g, out, stats, bn, before_finalize)
    bm, bn_ = tile or fwd_tile(g, Nb, x.dtype, pro is not None, Kpad)
    d = g.desc(Nb)
    # direct (unstaged) f32 store + bias: the fc head (16-bit features -> f32 logits, or any conv
    # with a bias); f32 activations of the exact-fp32 engine take the staged path with statistics
    out_f32 = bias is not None or out.dtype != x.dtype
    pitch = out.stride(0) if out.dim() == 2 else g.Cout
    kdt = _kdt(x)
    kbm, kbn = _ktile(bm, bn_, kdt, pro is not None or g.Cin < 64)
    T = math.ceil(M / tile_rows(kbm))
    if bn is not None:
        stats = bn.ws.get("fwd_stats", T * 3 * g.Cout)
    rc = ext.lib().pda_conv_fwd(C.byref(d), ptr(x), ptr(w), Kpad, ptr(out), int(out_f32), pitch,
                                ptr(bias), ptr(stats), int(relu), ptr(pro[0] if pro else None),
                                ptr(pro[1] if pro else None), kdt, kbm, kbn, stream(x.device))
    check(rc, "conv_fwd")
    if before_finalize is not None:
        before_finalize()
    if bn is not None:
        bn_finalize_partials(stats, T, g.Cout, tile_rows(kbm), M, bn)
    return out


@dataclass
class TailIn:
    """Operands of a residual block's tail a = relu(y3 * sc + sh + r) formed by the consumer conv
    (conv_fwd ``tail``): ``res`` is r itself (identity shortcut) or, with ``sc2`` / ``sh2``, the
    downsample branch's pre-BN output whose BN is applied too; ``out`` receives a, ``mask`` (uint8,
    numel / 8, identity tails) its ReLU bitmask -- exactly what :func:`bn_apply` would write."""
    res: torch.Tensor
    out: torch.Tensor
    mask: Optional[torch.Tensor] = None
    sc2: Optional[torch.Tensor] = None
    sh2: Optional[torch.Tensor] = None


def tail_fuse_ok(g: ConvGeom, dtype: torch.dtype) -> bool:
    """Whether a tail can be folded into this consumer conv (csrc/conv_gemm.hip FWD_TAIL): a 1x1
    stride-1 conv without padding on 16-bit operands, Cin a multiple of 64."""
    return (dtype in (torch.bfloat16, torch.float16) and g.R == 1 and g.S == 1 and g.stride == 1
            and g.pad == 0 and g.Cin % 64 == 0
            and getattr(ext.lib(), "pda_conv_fwd_tail", None) is not None)


def _conv_fwd_tail(y3, w, g: ConvGeom, out, pro, tail: TailIn, stats, bn, before_finalize):
    if pro is None or not tail_fuse_ok(g, y3.dtype):
        raise ValueError("conv_fwd tail: needs pro = (scale, shift) of the tail BN and a 1x1 "
                         "stride-1 16-bit conv (tail_fuse_ok)")
    if tail.out.shape != y3.shape or tail.res.shape != y3.shape or tail.out.dtype != y3.dtype:
        raise ValueError("conv_fwd tail: y3, the residual and the output activation share one shape")
    if tail.mask is not None and tail.mask.numel() * 8 < y3.numel():
        raise ValueError("conv_fwd tail: mask needs numel / 8 bytes")
    Nb = y3.shape[0]
    M = Nb * g.Ho * g.Wo
    Kpad = w.shape[-1] if w.dim() == 2 else w[0].numel()
    bm, bn_ = -128, (64 if g.Cout <= 64 else 128)
    T = math.ceil(M / 128)
    if bn is not None:
        stats = bn.ws.get("fwd_stats", T * 3 * g.Cout)
    mode = 2 if tail.sc2 is not None else 1
    d = g.desc(Nb)
    check(ext.lib().pda_conv_fwd_tail(C.byref(d), ptr(y3), ptr(w), Kpad, ptr(out), ptr(stats),
                                      ptr(pro[0]), ptr(pro[1]), ptr(tail.res), ptr(tail.sc2),
                                      ptr(tail.sh2), ptr(tail.out), ptr(tail.mask), mode,
                                      _kdt(y3), bm, bn_, stream(y3.device)), "conv_fwd_tail")
    if before_finalize is not None:
        before_finalize()
    if bn is not None:
        bn_finalize_partials(stats, T, g.Cout, 128, M, bn)
    return out


_STEM_FWD = True   # the stem conv on csrc/stem.hip (False: the generic 128x64 tile, tests)
# persistent blocks of the stem kernel: 256 / 512 / 1024 / 2048 measured 305 / 267 / 258 / 278 us
# (profiles/ab_r4.md section 15); 0 = the kernel's default, 1024
_STEM_GRID = 0


def stem_fwd_ok(g: ConvGeom, dtype: torch.dtype) -> bool:
    """Whether the space-to-depth stem conv (4x4/1, pad 2 top/left, 16 -> 64 channels) runs on the
    dedicated tap-reuse kernel (csrc/stem.hip): 16-bit, H % 4 == 0, W % 16 == 0, W <= 128."""
    return (_STEM_FWD and dtype in (torch.bfloat16, torch.float16) and g.R == 4 and g.S == 4
            and g.Cin == 16 and g.Cout == 64 and g.stride == 1 and g.pad == 2 and g.Ho == g.H
            and g.Wo == g.W and g.H % 4 == 0 and g.W % 16 == 0 and 16 <= g.W <= 128
            and getattr(ext.lib(), "pda_stem_fwd", None) is not None)


def stem_fwd(x: torch.Tensor, w: torch.Tensor, g: ConvGeom, out: torch.Tensor,
             stats: Optional[torch.Tensor] = None, bn: Optional[BnStats] = None,
             before_finalize=None) -> torch.Tensor:
    """The stem conv on csrc/stem.hip (input slab staged once per 4-row tile in LDS, taps read
    from it; persistent blocks keep the 64 x 256 weights in LDS). Statistics: shifted partials over
    output rows, the format :func:`bn_finalize_partials` / :func:`stats_totals` take
    (pass ``bm = stem_stats_rows(g)``)."""
    Nb = x.shape[0]
    M = Nb * g.Ho * g.Wo
    rows = stem_stats_rows(g)
    T = M // rows
    if bn is not None:
        stats = bn.ws.get("fwd_stats", T * 3 * g.Cout)
    if stats is not None and stats.numel() < T * 3 * g.Cout:
        raise ValueError(f"stem_fwd: stats needs {T * 3 * g.Cout} floats (one partial per output "
                         f"row, stem_stats_rows), got {stats.numel()}")
    check(ext.lib().pda_stem_fwd(ptr(x), ptr(w), ptr(out), ptr(stats), Nb, g.H, g.W, _kdt(x),
                                 _STEM_GRID, stream(x.device)), "stem_fwd")
    if before_finalize is not None:
        before_finalize()
    if bn is not None:
        bn_finalize_partials(stats, T, g.Cout, rows, M, bn)
    return out


def stem_stats_rows(g: ConvGeom) -> int:
    """Rows of M per statistics tile of :func:`stem_fwd` (one output row)."""
    return g.Wo


def stats_totals(stats: torch.Tensor, M: int, C_: int, bm: int) -> torch.Tensor:
    """f64 [2][C] (sum y, sum y^2) from conv_fwd's shifted per-tile partials (tests, tools)."""
    T = math.ceil(M / tile_rows(bm))
    p = stats[:T * 3 * C_].view(T, 3, C_).double()
    rows = torch.full((T, 1), float(tile_rows(bm)), dtype=torch.float64, device=stats.device)
    rows[-1, 0] = M - (T - 1) * tile_rows(bm)
    d0, d1, sh = p[:, 0], p[:, 1], p[:, 2]
    return torch.stack([(rows * sh + d0).sum(0), (d1 + sh * (2 * d0 + rows * sh)).sum(0)])


def bn_finalize_partials(stats: torch.Tensor, T: int, C_: int, bm: int, M: int, bn: BnStats) -> None:
    """BatchNorm forward statistics from conv_fwd's shifted per-tile partials in one launch
    (csrc/bn.hip bn_stats_kernel<0>): S blocks per 256-channel group reduce tile ranges to f64 slabs,
    the group's last arriving block sums them and finalizes. SyncBatchNorm (``ws.sync_comm``): the
    launch stops at f64 totals, which are all-reduced before :func:`bn_finalize_tot`."""
    G = math.ceil(C_ / _stats_cg(C_))
    S = _stats_slabs(T, C_)
    ws = bn.ws
    slabs = ws.get("bn_slabs", S * 2 * C_, torch.float64)
    cnt = ws.counters(G)
    sync = getattr(ws, "sync_comm", None)
    if sync is not None and sync.world_size == 1:
        sync = None
    tot = ws.get("bn_tot", 2 * C_, torch.float64) if sync is not None else None
    o = ext.BnFwdOut(ptr(bn.gamma), ptr(bn.beta), bn.eps, bn.momentum, ptr(bn.mean),
                     ptr(bn.invstd), ptr(bn.scale), ptr(bn.shift), ptr(bn.rmean), ptr(bn.rvar),
                     ptr(bn.nbt), int(bn.update), ptr(tot))
    check(ext.lib().pda_bn_fwd_stats(ptr(stats), T, C_, bm, M, S, ptr(slabs), ptr(cnt), C.byref(o),
                                     _stats_cg(C_), stream(stats.device)), "bn_fwd_stats")
    if sync is not None:   # SyncBatchNorm: global f64 totals, then finalize
        sync.all_reduce(tot)
        bn_finalize_tot(tot, C_, M * sync.world_size, bn)


def bn_finalize_tot(tot: torch.Tensor, C_: int, count: int, bn: BnStats) -> None:
    rc = ext.lib().pda_bn_finalize_tot(ptr(tot), C_, float(count), ptr(bn.gamma), ptr(bn.beta),
                                       bn.eps, bn.momentum, ptr(bn.mean), ptr(bn.invstd),
                                       ptr(bn.scale), ptr(bn.shift), ptr(bn.rmean), ptr(bn.rvar),
                                       ptr(bn.nbt), int(bn.update), stream(tot.device))
    check(rc, "bn_finalize_tot")


def stats_tiles(M: int, Cout: int, tile: Optional[Tuple[int, int]] = None) -> int:
    bm, _ = tile or pick_tile(M, Cout)
    return math.ceil(M / tile_rows(bm))


def _halo_geom(g: ConvGeom) -> bool:
    """3x3 / stride 1 / pad 1 convolutions whose input rows fit the tap-reuse slab (W <= 63)."""
    return (g.R == 3 and g.S == 3 and g.stride == 1 and g.pad == 1 and g.W <= 63
            and g.Cin % 64 == 0 and g.Cout % 64 == 0)


def dgrad_tile(g: ConvGeom, Nb: int, dma: bool = True) -> Tuple[int, int]:
    """Data-gradient tile: the tap-reuse (HALO) 256x128 LDS-DMA tile for 3x3 stride-1 layers with
    >= 128 channels (``PDA_DGRAD_HALO``; round 3 measured it slower in the step, 28.03 -> 27.88
    ms/step without it, profiles/ab_r3_dma.md section 11; with the round-4 MFMA-burst priority it
    wins, profiles/ab_r4.md section 17), the register-staged tiles otherwise. ``dma``: 16-bit
    operands (the DMA tiles need them)."""
    if dma and _DMA and _DGRAD_HALO and _halo_geom(g) and g.Cin >= 128:
        return 2256, 128
    M = Nb * (g.H // g.stride) * (g.W // g.stride)
    return pick_tile(M * g.stride * g.stride, g.Cin, g.Cout * _max_class_taps(g))


# the HALO data-gradient tile in the step: slower in round 3; with this round's raised-priority
# MFMA bursts (profiles/ab_r4.md section 11) -0.03 ms/step over 7 in-step pairs (section 17)
_DGRAD_HALO = os.environ.get("PDA_DGRAD_HALO", "1") != "0"


def _max_class_taps(g: ConvGeom) -> int:
    if g.stride == 1:
        return g.R * g.S
    return max(sum(1 for r in range(g.R) if (ph + g.pad - r) % 2 == 0) *
               sum(1 for s in range(g.S) if (pw + g.pad - s) % 2 == 0)
               for ph in (0, 1) for pw in (0, 1))


def dgrad_slabs(g: ConvGeom, Nb: int, tile: Optional[Tuple[int, int]] = None,
                dtype: Optional[torch.dtype] = None) -> int:
    """Number of partial-sum slabs the fused BN epilogue of a dgrad writes (classes x M-tiles);
    ``dtype`` = the dgrad's operand dtype (the tile it launches may differ: :func:`_ktile`)."""
    kdt = 1 if dtype is None else _kdt(torch.empty(0, dtype=dtype))
    bm, bn = tile or dgrad_tile(g, Nb, dma=kdt in (1, 2))
    bm, _ = _ktile(bm, bn, kdt)
    M = Nb * (g.H // g.stride) * (g.W // g.stride)
    return g.stride * g.stride * math.ceil(M / tile_rows(bm))


def conv_dgrad(dy: torch.Tensor, w: torch.Tensor, g: ConvGeom, dx: torch.Tensor,
               tile: Optional[Tuple[int, int]] = None, epi: Optional[ext.BnEpi] = None) -> torch.Tensor:
    """dx[Nb,H,W,Cin] = conv_transpose(dy[Nb,Ho,Wo,Cout], w[Cout,R,S,Cin]).

    With ``epi`` (see :func:`bn_epilogue`) the kernel instead stores dz = dA * relu_mask (dA = the
    transposed conv result [+ epi.g2]) and writes the BatchNorm-backward partial sums."""
    Nb = dy.shape[0]
    kdt = _kdt(dy)
    bm, bn = tile or dgrad_tile(g, Nb, dma=kdt in (1, 2))
    d = g.desc(Nb)
    kbm, kbn = _ktile(bm, bn, kdt)
    rc = ext.lib().pda_conv_dgrad(C.byref(d), ptr(dy), ptr(w), ptr(dx),
                                  C.byref(epi) if epi is not None else None, kdt, kbm, kbn,
                                  stream(dy.device))
    check(rc, "conv_dgrad")
    return dx


def bn_fold(w: torch.Tensor, k: torch.Tensor, wf: torch.Tensor, bias: torch.Tensor,
            ws: Optional["Workspace"] = None) -> None:
    """Operands of :func:`conv_dgrad_bnf` for a 1x1 conv (``w`` 16-bit [Cout, Cin], ``k`` =
    [k1; k2; k3] 3 x Cout f32 of the BatchNorm after it): ``wf`` [Cout + Cin, Cin] = [k1 o W ;
    W^T diag(k2) W], ``bias`` [Cin] = W^T k3 (csrc/conv_gemm.hip bn_fold_kernel, one launch;
    ``ws`` is accepted for call-site symmetry and unused)."""
    Cout, Cin = w.shape[0], w.shape[-1]
    if wf.shape[0] != Cout + Cin or wf.shape[-1] != Cin or wf.dtype != w.dtype or k.numel() < 3 * Cout:
        raise ValueError("bn_fold: wf [Cout + Cin, Cin] of the weights' dtype, k 3 x Cout")
    check(ext.lib().pda_bn_fold(ptr(w), ptr(k), Cout, Cin, ptr(wf), ptr(bias), dt_of(w),
                                stream(w.device)), "bn_fold")


def bnf_ok(g: ConvGeom, dtype: torch.dtype) -> bool:
    """Whether the consumer-side BN-backward fold (:func:`conv_dgrad_bnf`) serves this conv: a 1x1
    conv without padding, 16-bit operands, channel counts in whole 64-column panels."""
    return (g.R == 1 and g.S == 1 and g.pad == 0 and dtype in (torch.bfloat16, torch.float16)
            and g.Cin % 64 == 0 and g.Cout % 64 == 0
            and getattr(ext.lib(), "pda_conv_dgrad_bnf", None) is not None)


def conv_dgrad_bnf(dz: torch.Tensor, wf: torch.Tensor, g: ConvGeom, dx: torch.Tensor,
                   xa: torch.Tensor, bias: torch.Tensor, xa_pro=None,
                   epi: Optional[ext.BnEpi] = None,
                   tile: Optional[Tuple[int, int]] = None) -> torch.Tensor:
    """dX of a 1x1 conv whose dY = k1*dz + k2*y + k3 is never materialised (y = the conv's forward
    output): dX = dz . (k1 o W) + xa . G + b with (wf, bias) from :func:`bn_fold` and ``xa`` the
    conv's forward input (``xa_pro`` = (scale, shift): xa is PRE-BatchNorm and the activation
    relu(xa*scale+shift) is recomputed, as the forward's prologue did). ``epi``: the same fused
    BN-backward epilogue as :func:`conv_dgrad`."""
    Nb = dz.shape[0]
    kdt = _kdt(dz)
    bm, bn = tile or dgrad_tile(g, Nb)
    kbm, kbn = _ktile(bm, bn, kdt)
    if kbm > 1000:    # the fold's Gram operand needs the register-staged loader
        kbm, kbn = -128, min(kbn, 128)
    d = g.desc(Nb)
    rc = ext.lib().pda_conv_dgrad_bnf(C.byref(d), ptr(dz), ptr(wf), ptr(dx),
                                      C.byref(epi) if epi is not None else None, ptr(xa),
                                      ptr(xa_pro[0] if xa_pro else None),
                                      ptr(xa_pro[1] if xa_pro else None), ptr(bias),
                                      kdt, kbm, kbn, stream(dz.device))
    check(rc, "conv_dgrad_bnf")
    return dx


def bn_epilogue(ws: "Workspace", G: int, y, scale, shift, res=None, y2=None, scale2=None,
                shift2=None, g2=None, mask=None):
    """Describe the BN-backward reduction a dgrad epilogue performs for a = relu(bn(y) [+res | +bn2(y2)]).
    ``mask`` (the forward's ReLU bitmask of a, see :func:`bn_apply`) replaces ``res``: the epilogue
    then reads one byte per 8 elements instead of the residual tensor (mode 3).
    Returns (epi, part, nq): ``part`` holds G*nq*C partials after the dgrad (:func:`bn_bwd_finish`
    finalizes them)."""
    C_ = y.shape[-1]
    mode = 3 if mask is not None else (2 if y2 is not None else (1 if res is not None else 0))
    nq = 3 if mode == 2 else 2
    part = ws.get("bn_part", G * nq * C_)
    epi = ext.BnEpi(mode, nq, ptr(y), ptr(scale), ptr(shift),
                    ptr(y2 if y2 is not None else res), ptr(scale2), ptr(shift2), ptr(g2), ptr(part),
                    ptr(mask))
    return epi, part, nq


# Weight-gradient tile / split-K block target per ResNet conv geometry (Cout, R, Cin, stride, Ho),
# measured on MI355X at batch 400: tools/wgrad_sweep.py (profiles/wgrad_sweep_r1_v2.txt), then
# tools/conv_bench.py re-measurements (profiles/convbench_r2.txt; round 3: the LDS-DMA 8-wave tiles,
# 1000 + rows, win on the 3x3 and strided weight gradients, profiles/convbench_r3_dma.txt).
_WGRAD_TUNED = {
    (64, 1, 64, 1, 56): ((-64, 128), 512),      # C1
    (64, 3, 64, 1, 56): ((64, 128), 512),       # C2
    (256, 1, 64, 1, 56): ((-128, 64), 512),     # C3 (round 5, decomposed conv3 fold: -128x128 +0.05 ms)
    (64, 1, 256, 1, 56): ((128, 128), 512),     # C4
    (128, 1, 256, 1, 56): ((-128, 128), 512),   # C5
    (128, 3, 128, 2, 28): ((128, 64), 2048),    # C6
    (512, 1, 128, 1, 28): ((128, 128), 512),    # C7
    (512, 1, 256, 2, 28): ((-256, 128), 512),   # C8
    (128, 1, 512, 1, 28): ((-128, 128), 512),   # C9
    (128, 3, 128, 1, 28): ((-64, 128), 512),    # C10
    (256, 1, 512, 1, 28): ((-256, 128), 1024),  # C11
    (256, 3, 256, 2, 14): ((-256, 128), 512),   # C12
    (1024, 1, 256, 1, 14): ((-128, 128), 512),  # C13 (round 5: -0.17 ms/step vs -128x64, ab_r5.md s.14)
    (1024, 1, 512, 2, 14): ((128, 128), 512),   # C14
    (256, 1, 1024, 1, 14): ((-128, 64), 512),   # C15
    (256, 3, 256, 1, 14): ((-256, 128), 2048),  # C16
    (512, 1, 1024, 1, 14): ((128, 128), 512),   # C17
    (512, 3, 512, 2, 7): ((-256, 128), 4096),   # C18
    (2048, 1, 512, 1, 7): ((-128, 128), 512),   # C19
    (2048, 1, 1024, 2, 7): ((-128, 128), 512),  # C20
    (512, 1, 2048, 1, 7): ((128, 128), 512),    # C21
    (512, 3, 512, 1, 7): ((-256, 128), 1024),   # C22
    # stem (4x4/1 on the space-to-depth image, WGRAD_BNA): the 64x256 tile (the whole N: dz and y
    # staged once) at ~1024 splits, 404 us vs 440 for 64x128 at 1536 blocks and 490 at the 512
    # default -- it runs alone at the end of the backward (tools/stem_wgrad_sweep.py)
    (64, 4, 16, 1, 112): ((-64, 256), 1536),
}
_WGRAD_ALONE = {(64, 4, 16, 1, 112)}   # weight gradients with nothing beside them (no x0.7)
# LDS-DMA tiles (16-bit, no operand prologue; the register-staged entry above is the fallback)
_DMA = os.environ.get("PDA_DMA", "1") != "0"
_WGRAD_DMA = {   # tools/wgrad_sweep.py, kernel + slab reduce (profiles/wgrad_sweep_r3{,b}.txt)
    (256, 1, 64, 1, 56): ((1256, 128), 256),    # C3  159 -> 153 us (the downsample; conv3: prologue)
    (64, 1, 256, 1, 56): ((1128, 256), 256),    # C4  160 -> 151
    (128, 1, 256, 1, 56): ((1128, 256), 256),   # C5  206 -> 182
    (128, 3, 128, 2, 28): ((1128, 256), 512),   # C6  200 -> 200 (conv_bench: 221 -> 197)
    (512, 1, 128, 1, 28): ((1256, 128), 256),   # C7  113 ->  98
    (512, 1, 256, 2, 28): ((1256, 256), 512),   # C8  168 -> 137
    (128, 1, 512, 1, 28): ((1128, 256), 256),   # C9  115 ->  96
    (128, 3, 128, 1, 28): ((1128, 256), 512),   # C10 171 -> 168
    (256, 1, 512, 1, 28): ((1256, 256), 256),   # C11 165 -> 140
    (256, 3, 256, 2, 14): ((1256, 256), 512),   # C12 171 -> 124
    (1024, 1, 512, 2, 14): ((1256, 256), 512),  # C14 133 -> 121
    (256, 1, 1024, 1, 14): ((1256, 256), 256),  # C15  78 ->  75
    (256, 3, 256, 1, 14): ((1256, 256), 256),   # C16 161 -> 120
    (512, 1, 1024, 1, 14): ((1256, 256), 256),  # C17 130 -> 122
    (512, 3, 512, 2, 7): ((1256, 256), 512),    # C18 134 -> 119
    (2048, 1, 512, 1, 7): ((1128, 256), 256),   # C19  67 ->  60
    (2048, 1, 1024, 2, 7): ((1256, 256), 512),  # C20 118 -> 111
    (512, 1, 2048, 1, 7): ((1256, 128), 256),   # C21  70 ->  61
    (512, 3, 512, 1, 7): ((1256, 256), 512),    # C22 129 -> 116
}


def wgrad_plan(g: ConvGeom, Nb: int, tile: Optional[Tuple[int, int]] = None,
               target_blocks: Optional[int] = None, max_slab_bytes: int = 64 << 20,
               f32: bool = False, dma: bool = False, wscale: Optional[float] = None,
               bna: bool = False):
    """(bm, bn, splits, k_chunk) of a weight gradient; ``dma``: the launch may use an LDS-DMA tile
    (16-bit operands, no operand prologue); ``wscale``: the split-K block-target factor of the
    caller's schedule (None: ``PDA_WGRAD_SCALE``, the concurrent eager step's x0.7)."""
    M, N, K = g.Cout, g.R * g.S * g.Cin, Nb * g.Ho * g.Wo
    key = (g.Cout, g.R, g.Cin, g.stride, g.Ho)
    tuned = _WGRAD_TUNED.get(key)
    if dma and _DMA and key in _WGRAD_DMA:
        tuned = _WGRAD_DMA[key]
    bn = 128 if N >= 128 else 64
    bm = 128 if M >= 128 else 64
    if bm == 128 or bn == 128:
        bm = -bm      # single-LDS-buffer variants (tools/conv_bench.py: best or within 2%)
    if tuned and not tile:
        (bm, bn), tb = tuned
        target_blocks = target_blocks or tb
        if f32 and (tile_rows(bm) > 128 or bn > 128):   # 256-wide tiles are 16-bit only
            bm, bn = -128, 128
        if bna and (abs(bm), bn) not in _BNA_TILES:     # the nearest tile WGRAD_BNA is built for
            bm, bn = -128, 128
        if bna and M <= 64 and tile_rows(bm) > 64:        # Cout 64 (the layer1 conv1): no idle rows
            bm, bn = -64, 128
    if target_blocks is None:
        target_blocks = _WGRAD_TARGET
    # (the stem's weight gradient runs alone at the end of the backward: its isolated optimum holds)
    sc = _WGRAD_SCALE if wscale is None else wscale
    target_blocks = max(1, int(target_blocks * (1.0 if key in _WGRAD_ALONE else sc)))
    if tile:
        bm, bn = tile
    tiles = math.ceil(M / tile_rows(bm)) * math.ceil(N / bn)
    splits = max(1, min(math.ceil(target_blocks / tiles), math.ceil(K / 256),
                        max(1, max_slab_bytes // (M * N * 4))))
    k_chunk = math.ceil(K / splits / 64) * 64
    splits = math.ceil(K / k_chunk)
    return bm, bn, splits, k_chunk


def wgrad_bna_ok(g: ConvGeom, Nb: int, dtype: torch.dtype) -> bool:
    """Whether :func:`conv_wgrad` can form dY from the BN backward in-kernel for this geometry: 16-bit
    operands on the tiles WGRAD_BNA is built for (64x128, 64x256: the stem's Cout = 64)."""
    if dtype not in (torch.bfloat16, torch.float16) or g.Cout % 8:
        return False
    if getattr(ext.lib(), "pda_conv_wgrad_bna", None) is None:
        return False
    bm, bn, _, _ = wgrad_plan(g, Nb, bna=True)
    return (abs(bm), bn) in _BNA_TILES


# tiles pda_conv_wgrad_bna is built for (csrc/conv_gemm.hip BNA_CASE): the stem's 64-row tiles and
# the bottleneck conv3 weight gradients of the consumer-side tail fold
_BNA_TILES = {(64, 128), (64, 256), (128, 128), (128, 64)}


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, g: ConvGeom, grad: torch.Tensor, ws: Workspace,
               cin_real: Optional[int] = None, scale: float = 1.0, accumulate: bool = False,
               tile: Optional[Tuple[int, int]] = None,
               pro: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
               target_blocks: Optional[int] = None,
               bna: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
               wscale: Optional[float] = None,
               combine: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """grad (f32, OHWI with cin_real channels, rows of pitch R*S*cin_real) = scale * dW.
    pro = (scale, shift): x is PRE-BatchNorm; the activation relu(x*scale+shift) is recomputed.
    bna = (y, k) with k = [k1; k2; k3] (3 x Cout f32): ``dy`` is the BN-backward's masked gradient
    dz and the kernel stages dY = k1*dz + k2*y + k3 itself (csrc/conv_gemm.hip WGRAD_BNA; see
    :func:`wgrad_bna_ok`).
    combine = (k, B, s): the decomposed form of that weight gradient -- ``dy`` is dz, the GEMM is
    the plain dz^T x, and the split-K reduce writes k1*(dz^T x) + k2*B + k3*s^T per row, with
    B = W Gram(x) and s the column sums of x (:func:`conv_wgrad_gram`, :func:`fold_bgemm`)."""
    Nb = dy.shape[0]
    if (tile is None and target_blocks is None and bna is None and combine is None
            and cin_real is None and wgrad_tap_ok(g, dy.dtype)):
        return conv_wgrad_tap(dy, x, g, grad, ws, scale, accumulate, pro)
    if (tile is None and target_blocks is None and bna is not None and combine is None
            and cin_real is None and pro is None and stem_wgrad_tap_ok(g, dy.dtype)):
        return conv_wgrad_stem_tap(dy, bna[0], bna[1], x, g, grad, ws, scale, accumulate)
    bm, bn, splits, k_chunk = wgrad_plan(g, Nb, tile, target_blocks, f32=dy.dtype == torch.float32,
                                         dma=dy.dtype != torch.float32 and pro is None and bna is None,
                                         wscale=wscale, bna=bna is not None)
    if bna is None and bm == -64 and bn == 256:
        # 64x256 is a WGRAD_BNA tile: the plain weight gradient of that plan runs 64x128 tiles over
        # the same split-K chunks (same accumulation order per element: bitwise the same result)
        bn = 128
    M, N = g.Cout, g.R * g.S * g.Cin
    rb = ws.reduce_batch if N % 4 == 0 else None
    slab = rb.slab(splits * M * N) if rb is not None else ws.get("wgrad_slab", splits * M * N)
    d = g.desc(Nb)
    st = stream(dy.device)
    kdt = _kdt(dy)
    kbm, kbn = _ktile(bm, bn, kdt)
    if bna is not None:
        y, k = bna
        Co = g.Cout
        rc = ext.lib().pda_conv_wgrad_bna(C.byref(d), ptr(dy), ptr(y), ptr(k[0:Co]), ptr(k[Co:2 * Co]),
                                          ptr(k[2 * Co:3 * Co]), ptr(x), ptr(slab), splits, k_chunk,
                                          ptr(pro[0] if pro else None), ptr(pro[1] if pro else None),
                                          kdt, kbm, kbn, st)
        check(rc, "conv_wgrad_bna")
    else:
        rc = ext.lib().pda_conv_wgrad(C.byref(d), ptr(dy), ptr(x), ptr(slab), splits, k_chunk,
                                      ptr(pro[0] if pro else None), ptr(pro[1] if pro else None),
                                      kdt, kbm, kbn, st)
        check(rc, "conv_wgrad")
    cr = g.Cin if cin_real is None else cin_real
    ck, cB, cs = combine if combine is not None else (None, None, None)
    if rb is not None:
        rb.add(slab, grad, splits, M, N, int(math.log2(g.Cin)), cr, g.R * g.S * cr, scale,
               accumulate, ck, cB, cs)
        return grad
    rc = ext.lib().pda_wgrad_reduce(ptr(slab), ptr(grad), splits, M, N, int(math.log2(g.Cin)), cr,
                                    g.R * g.S * cr, float(scale), int(accumulate), ptr(ck), ptr(cB),
                                    ptr(cs), st)
    check(rc, "wgrad_reduce")
    return grad


# which 3x3 stride-1 weight gradients run the tap-reuse kernel (csrc/wgrad_tap.hip), by image width
# ("0": none); the generic tiles re-read X per (tap, channel) column tile and dY per N-tile
_WGRAD_TAP = {int(v) for v in os.environ.get("PDA_WGRAD_TAP", "56,28").replace("+", ",").split(",")
              if v.strip() not in ("", "0")}
# blocks of the tap-reuse weight gradient (one 104 KiB block per CU: the split count is the block
# count). Alone 256 is fastest (C2 165 vs 176 us at 512); in the step fewer blocks leave the other
# CUs to the main chain: 256 / 192 / 128 / 112 / 96 / 80 / 64 -> 96 (-0.2 ms/step vs 256;
# profiles/ab_r5.md section 15)
_WGRAD_TAP_BLOCKS = int(os.environ.get("PDA_WGRAD_TAP_BLOCKS", "96"))


def wgrad_tap_ok(g: ConvGeom, dtype: torch.dtype) -> bool:
    """Whether :func:`conv_wgrad` runs the tap-reuse kernel for this conv: 3x3 / stride 1 / pad 1,
    16-bit, channel counts in 64-column tiles, image width in the ``PDA_WGRAD_TAP`` set (<= 59).
    Cin must be a power of two: the reduce decodes a slab column's tap as ``n >> log2(Cin)``."""
    return (dtype in (torch.bfloat16, torch.float16) and g.R == 3 and g.S == 3 and g.stride == 1
            and g.pad == 1 and g.Ho == g.H and g.Wo == g.W and g.W <= 59 and g.W in _WGRAD_TAP
            and g.Cin % 64 == 0 and g.Cout % 64 == 0 and (g.Cin & (g.Cin - 1)) == 0
            and getattr(ext.lib(), "pda_wgrad_tap", None) is not None)


def wgrad_tap_plan(g: ConvGeom, Nb: int, blocks: int = _WGRAD_TAP_BLOCKS) -> Tuple[int, int]:
    """(kb, splits): padded pixel rows per split (a multiple of 64) and the split count of the
    tap-reuse weight gradient for ~``blocks`` blocks over its (Cout / 64) x (Cin / 64) tiles."""
    kp = Nb * (g.H + 2) * (g.W + 2)
    tiles = (g.Cout // 64) * (g.Cin // 64)
    want = max(1, blocks // tiles)
    kb = max(64, math.ceil(kp / want / 64) * 64)
    return kb, math.ceil(kp / kb)


def conv_wgrad_tap(dy: torch.Tensor, x: torch.Tensor, g: ConvGeom, grad: torch.Tensor,
                   ws: "Workspace", scale: float = 1.0, accumulate: bool = False,
                   pro: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """grad (f32 OHWI) = scale * dW of a 3x3 stride-1 conv on the tap-reuse kernel: each block
    loads its pixel range of dY and X once for all nine taps (csrc/wgrad_tap.hip), split-K slabs
    reduced by the same fixed-order launch as :func:`conv_wgrad`. ``pro`` as there."""
    Nb = dy.shape[0]
    kb, splits = wgrad_tap_plan(g, Nb)
    M, N = g.Cout, 9 * g.Cin
    rb = ws.reduce_batch
    slab = rb.slab(splits * M * N) if rb is not None else ws.get("wgrad_slab", splits * M * N)
    st = stream(dy.device)
    L = ext.lib()
    check(L.pda_wgrad_tap(ptr(dy), ptr(x), ptr(slab), ptr(pro[0] if pro else None),
                          ptr(pro[1] if pro else None), Nb, g.H, g.W, g.Cin, g.Cout, kb, splits,
                          _kdt(dy), st), "wgrad_tap")
    if rb is not None:
        rb.add(slab, grad, splits, M, N, int(math.log2(g.Cin)), g.Cin, N, scale, accumulate)
        return grad
    check(L.pda_wgrad_reduce(ptr(slab), ptr(grad), splits, M, N, int(math.log2(g.Cin)), g.Cin, N,
                             float(scale), int(accumulate), None, None, None, st), "wgrad_reduce")
    return grad


# PDA_STEM_WGRAD=tap: the stem's weight gradient (WGRAD_BNA operand) on the tap-reuse kernel
# (csrc/wgrad_tap.hip wgrad_stem_tap_kernel) instead of the implicit-GEMM WGRAD_BNA 64x256 tile.
# Off by default: 368-381 us vs 375-380 us alone at batch 400, step time unchanged within noise
# (profiles/ab_r6.md section 15). Blocks = splits (one 113 KiB block per CU)
_STEM_WGRAD = os.environ.get("PDA_STEM_WGRAD", "generic")
_STEM_TAP_BLOCKS = int(os.environ.get("PDA_STEM_TAP_BLOCKS", "512"))


# Events that order the second stream after the main one (fork tracking's per-launch completion
# event, the DataParallel replay's side-graph hand-offs). PDA_EVENT_SYSFENCE=1: HIP's default event,
# whose completion carries a SYSTEM-scope release (a full L2 write-back, for host / peer
# visibility); 0: hipEventDisableSystemFence -- only a stream of the same device waits on these,
# for which the agent-scope release of the kernel's own completion is enough.
_EVENT_SYSFENCE = os.environ.get("PDA_EVENT_SYSFENCE", "1") == "1"


def fork_event_create():
    """A ``hipEvent_t`` (ctypes void pointer) for same-device stream ordering: timing disabled,
    system-scope fence per PDA_EVENT_SYSFENCE."""
    ev = C.c_void_p()
    flags = 0x2 | (0 if _EVENT_SYSFENCE else 0x20000000)   # hipEventDisableTiming | ...SystemFence
    check(ext.lib().pda_event_create_flags(C.byref(ev), flags), "pda_event_create_flags")
    return ev


def stem_wgrad_tap_ok(g: ConvGeom, dtype: torch.dtype, force: bool = False) -> bool:
    """The space-to-depth stem conv (4x4, stride 1, pad 2, 16 -> 64 channels, same-size output) in
    16 bit, with the tap-reuse stem kernel built (and selected, unless ``force``)."""
    return ((force or _STEM_WGRAD == "tap") and dtype in (torch.bfloat16, torch.float16) and g.R == 4
            and g.S == 4 and g.stride == 1 and g.pad == 2 and g.Cin == 16 and g.Cout == 64
            and g.Ho == g.H and g.Wo == g.W and g.W + 3 <= 122
            and getattr(ext.lib(), "pda_wgrad_stem_tap", None) is not None)


def conv_wgrad_stem_tap(dz: torch.Tensor, y: torch.Tensor, k: torch.Tensor, x: torch.Tensor,
                        g: ConvGeom, grad: torch.Tensor, ws: "Workspace", scale: float = 1.0,
                        accumulate: bool = False, blocks: Optional[int] = None) -> torch.Tensor:
    """grad (f32 [64][16 taps x 16]) = scale * dW of the stem conv with dY = k1*dz + k2*y + k3
    formed in LDS (:func:`conv_wgrad` ``bna``): each block loads its pixel range of dz, y and the
    input once for all 16 taps; split-K slabs reduced by the same fixed-order launch."""
    Nb = dz.shape[0]
    kp = Nb * (g.H + 3) * (g.W + 3)
    nb = blocks or _STEM_TAP_BLOCKS
    kb = max(64, math.ceil(kp / nb / 64) * 64)
    splits = math.ceil(kp / kb)
    M, N = 64, 256
    rb = ws.reduce_batch
    slab = rb.slab(splits * M * N) if rb is not None else ws.get("wgrad_slab", splits * M * N)
    st = stream(dz.device)
    L = ext.lib()
    check(L.pda_wgrad_stem_tap(ptr(dz), ptr(y), ptr(k), ptr(x), ptr(slab), Nb, g.H, g.W, kb, splits,
                               _kdt(dz), st), "wgrad_stem_tap")
    if rb is not None:
        rb.add(slab, grad, splits, M, N, 4, 16, N, scale, accumulate)
        return grad
    check(L.pda_wgrad_reduce(ptr(slab), ptr(grad), splits, M, N, 4, 16, N, float(scale),
                             int(accumulate), None, None, None, st), "wgrad_reduce")
    return grad


_TAP_MASKS: Dict = {}


def stem_tap_colsum(x: torch.Tensor, g: ConvGeom) -> torch.Tensor:
    """f32 [R*S*Cin] (column t*Cin + ci, t = r*S + s): the sum over every valid output pixel of
    the stem conv's tap-(r, s) input, X[n][oy + r - pad][ox + s - pad][ci] (zero outside) -- the
    k3 term of the decomposed stem weight gradient. Tap r sees input rows [r - pad, H - 1 + r - pad]
    clipped to the image, so each tap's sum is the image total minus its excluded border rows /
    columns (the first R-1-pad, the last pad) plus their corners: a few small reductions of x
    (slices only: no index tensors, no host copies after the first call), not a pass per tap."""
    Nb, H, W, Cin = x.shape
    R, S, pad = g.R, g.S, g.pad
    assert g.stride == 1 and g.Ho == H and g.Wo == W and H > 2 * R and W > 2 * S and pad < R
    nt, nb = R - 1 - pad, pad            # excluded top / bottom rows (and left / right columns)
    key = (H, W, R, S, pad, x.device)
    if key not in _TAP_MASKS:
        rows = list(range(nt)) + list(range(H - nb, H))
        cols = list(range(nt)) + list(range(W - nb, W))
        mr = [[0.0 if r - pad <= y <= H - 1 + r - pad else 1.0 for y in rows] for r in range(R)]
        mc = [[0.0 if q - pad <= c <= W - 1 + q - pad else 1.0 for c in cols] for q in range(S)]
        _TAP_MASKS[key] = (torch.tensor(mr, device=x.device), torch.tensor(mc, device=x.device))
    mr, mc = _TAP_MASKS[key]
    f32 = torch.float32
    tot = x.sum(dim=(0, 1, 2), dtype=f32)                                            # [Cin]
    rs = torch.cat([x[:, :nt].sum(dim=(0, 2), dtype=f32),
                    x[:, H - nb:].sum(dim=(0, 2), dtype=f32)])                       # [nr, Cin]
    cs = torch.cat([x[:, :, :nt].sum(dim=(0, 1), dtype=f32),
                    x[:, :, W - nb:].sum(dim=(0, 1), dtype=f32)])                    # [nc, Cin]
    q = torch.cat([torch.cat([x[:, :nt, :nt].sum(0, dtype=f32), x[:, :nt, W - nb:].sum(0, dtype=f32)], 1),
                   torch.cat([x[:, H - nb:, :nt].sum(0, dtype=f32),
                              x[:, H - nb:, W - nb:].sum(0, dtype=f32)], 1)])        # [nr, nc, Cin]
    out = (tot[None, None] - (mr @ rs)[:, None] - (mc @ cs)[None, :]
           + torch.einsum("ra,sb,abc->rsc", mr, mc, q))
    return out.reshape(-1).contiguous()


def conv_wgrad_gram(y: torch.Tensor, sc: torch.Tensor, sh: torch.Tensor, gram: torch.Tensor,
                    ws: "Workspace") -> None:
    """gram [C + 1][C]: rows 0..C-1 = a^T a, row C = the column sums of a = relu(y*sc + sh) (y
    16-bit NHWC, C channels; csrc/conv_gemm.hip WGRAD_GRAM: both operands staged through the
    BN+ReLU, the diagonal tiles stage one image for both; split-K slabs reduced in fixed order by
    one launch). The forward-time half of the decomposed tail-fold weight gradient
    (:func:`conv_wgrad` ``combine``)."""
    Nb, H, W, C_ = y.shape
    if gram.numel() < (C_ + 1) * C_ or gram.dtype != torch.float32:
        raise ValueError("conv_wgrad_gram: gram f32 [C + 1][C]")
    P = Nb * H * W
    bm, bn = (64, 64) if C_ <= 64 else (-128, 128)
    tiles = math.ceil(C_ / tile_rows(bm)) * math.ceil(C_ / bn)
    splits = max(1, min(math.ceil(2 * _NUM_CU / tiles), math.ceil(P / 256),
                        max(1, (64 << 20) // (C_ * (C_ + 1) * 4))))
    k_chunk = math.ceil(P / splits / 64) * 64
    splits = math.ceil(P / k_chunk)
    slab = ws.get("gram_slab", splits * C_ * (C_ + 1))
    d = ConvGeom(Nb, H, W, C_, C_, 1, 1, 1, 0).desc(Nb)
    st = stream(y.device)
    L = ext.lib()
    check(L.pda_conv_wgrad_gram(C.byref(d), ptr(y), ptr(sc), ptr(sh), ptr(slab), splits, k_chunk,
                                _kdt(y), bm, bn, st), "conv_wgrad_gram")
    check(L.pda_wgrad_reduce(ptr(slab), ptr(gram), splits, C_ + 1, C_, int(math.log2(C_)), C_, C_,
                             1.0, 0, None, None, None, st), "gram_reduce")


def fold_bgemm(w: torch.Tensor, gram: torch.Tensor, out: torch.Tensor) -> None:
    """out [Cout][C] f32 = W Gram (W 16-bit [Cout][C], the forward's weights)."""
    Cout, C_ = w.shape[0], w.shape[-1]
    check(ext.lib().pda_fold_bgemm(ptr(w), ptr(gram), Cout, C_, ptr(out), dt_of(w), stream(w.device)),
          "fold_bgemm")


# ------------------------------------------------------------------ batchnorm
_PRE_S = 96


def prereduce(part: torch.Tensor, G: int, QC: int, ws: Optional["Workspace"] = None):
    """[G][QC] partial slabs -> [S][QC] with S in [96, 512] (coalesced first stage; narrow layers
    get more slices so the stage fills the chip), so the per-channel finalize kernels never walk
    thousands of slabs serially. Returns (part, G)."""
    S = max(_PRE_S, min(512, 65536 // max(QC, 1)))   # enough blocks for narrow layers
    if G <= 2 * S:
        return part, G
    out = (ws.get("bn_pre", 512 * QC) if ws is not None
           else torch.empty(S * QC, dtype=torch.float32, device=part.device))
    s = ext.lib().pda_slab_reduce(ptr(part), G, QC, S, ptr(out), stream(part.device))
    if s < 0:
        raise RuntimeError("slab_reduce launch failed")
    return out, s


def _sync_sums(part: torch.Tensor, G: int, QC: int, ws: Optional["Workspace"]):
    """SyncBatchNorm: [G][QC] partials -> one [QC] row (own slab kernel, fixed order), summed over
    the ranks of ``ws.sync_comm`` (ordered on the current stream). Returns (part, G, world)."""
    comm = getattr(ws, "sync_comm", None)
    if comm is None or comm.world_size == 1:
        return part, G, 1
    tot = ws.get("bn_sync", QC)
    if ext.lib().pda_slab_reduce(ptr(part), G, QC, 1, ptr(tot), stream(part.device)) < 0:
        raise RuntimeError("slab_reduce launch failed")
    comm.all_reduce(tot)
    return tot, 1, comm.world_size


def bn_eval_coeffs(gamma, beta, rmean, rvar, eps, scale, shift) -> None:
    rc = ext.lib().pda_bn_eval_coeffs(ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), float(eps),
                                      gamma.numel(), ptr(scale), ptr(shift), stream(gamma.device))
    check(rc, "bn_eval_coeffs")


def bn_apply(y, scale, shift, out, res=None, y2=None, scale2=None, shift2=None, relu=True,
             mask=None):
    """out = act(bn(y) [+ res | + bn2(y2)]); mask (uint8, numel/8) optionally receives the output's
    ReLU bitmask (bit e of byte i: element 8i+e > 0)."""
    mode = 2 if y2 is not None else (1 if res is not None else 0)
    r2 = y2 if y2 is not None else res
    rc = ext.lib().pda_bn_apply(ptr(y), ptr(scale), ptr(shift), ptr(r2), ptr(scale2), ptr(shift2),
                                ptr(out), y.numel(), y.shape[-1], mode, int(relu), ptr(mask),
                                dt_of(y), stream(y.device))
    check(rc, "bn_apply")
    return out


def stem_pool(y, scale, shift, out, arg):
    N, H, W, C_ = y.shape
    Ho, Wo = out.shape[1], out.shape[2]
    rc = ext.lib().pda_stem_pool(ptr(y), ptr(scale), ptr(shift), ptr(out), ptr(arg), N, H, W, C_, Ho,
                                 Wo, dt_of(y), stream(y.device))
    check(rc, "stem_pool")
    return out


def maxpool_bwd(dout, arg, din, dout2=None):
    N, H, W, C_ = din.shape
    Ho, Wo = dout.shape[1], dout.shape[2]
    rc = ext.lib().pda_maxpool_bwd(ptr(dout), ptr(dout2), ptr(arg), ptr(din), N, H, W, C_, Ho, Wo,
                                   dt_of(din), stream(din.device))
    check(rc, "maxpool_bwd")
    return din


def tail_pool(y, scale, shift, out, res=None, y2=None, scale2=None, shift2=None):
    N, H, W, C_ = y.shape
    mode = 2 if y2 is not None else 1
    r2 = y2 if y2 is not None else res
    rc = ext.lib().pda_tail_pool(ptr(y), ptr(scale), ptr(shift), ptr(r2), ptr(scale2), ptr(shift2),
                                 ptr(out), N, H * W, C_, mode, dt_of(y), stream(y.device))
    check(rc, "tail_pool")
    return out


def stem_bwd_reduce(ws: "Workspace", dout, arg, y, scale, shift, dz_out, dout2=None):
    """Stem backward, one pass: max-pool gradient gather (``dout`` [+ ``dout2``] through the argmax
    bytes) -> ReLU mask of relu(bn(y)) -> ``dz_out`` -> BatchNorm-backward partial sums.
    Returns (part, G, nq) for :func:`bn_bwd_finish`."""
    N, H, W, C_ = y.shape
    Ho, Wo = dout.shape[1], dout.shape[2]
    G = max(1, min(_STEM_G, (N * H * W) // 512))   # gather-latency bound: more blocks than a reduce
    part = ws.get("bn_part", G * 2 * C_)
    rc = ext.lib().pda_stem_bwd_reduce(ptr(dout), ptr(dout2), ptr(arg), ptr(y), ptr(scale), ptr(shift),
                                       ptr(dz_out), ptr(part), G, N, H, W, C_, Ho, Wo, dt_of(y),
                                       stream(y.device))
    check(rc, "stem_bwd_reduce")
    return part, G, 2


def _reduce_blocks(rows: int, C_: int) -> int:
    tpr = min(C_ // 8, 256)
    rpi = 256 // tpr
    # aim for ~1024 blocks with >= 4 row iterations each
    return max(1, min(1024, rows // (rpi * 4) or 1))


def bn_bwd(ws: Workspace, y, mean, invstd, gamma, scale, shift, dgamma, dbeta, dy_out,
           g1=None, g2=None, gp=None, res=None, y2=None, mean2=None, invstd2=None, gamma2=None,
           scale2=None, shift2=None, dgamma2=None, dbeta2=None, dy2_out=None, dz_buf=None,
           no_mask: bool = False, gscale: float = 1.0, accumulate: bool = False) -> None:
    """Backward of  a = relu(bn(y) [+ res | + bn2(y2)])  w.r.t. y (and y2).

    The incoming gradient is ``g1 (+ g2)`` or, for the pooled head, ``gp[n][c] / HW``.
    Writes dgamma/dbeta (f32, * gscale, optionally accumulated) and dy_out (16-bit).
    With a residual (``res`` or ``y2``) the masked gradient dz is materialised in ``dz_buf``
    because it is also the gradient of the shortcut input."""
    N, H, W, C_ = y.shape
    rows = N * H * W
    mode = 3 if no_mask else (2 if y2 is not None else (1 if res is not None else 0))
    nq = 3 if mode == 2 else 2
    G = _reduce_blocks(rows, C_)
    part = ws.get("bn_part", G * nq * C_)
    a = BwdArgs(ptr(g1), ptr(g2), ptr(gp), H * W if gp is not None else 0,
                ptr(y), ptr(scale), ptr(shift),
                ptr(y2 if y2 is not None else res), ptr(scale2), ptr(shift2),
                mode, ptr(dz_buf), ptr(part), nq, rows, C_)
    st = stream(y.device)
    L = ext.lib()
    dt = dt_of(y)
    check(L.pda_bn_bwd_reduce(C.byref(a), G, dt, st), "bn_bwd_reduce")
    _bn_bwd_tail(ws, part, G, nq, mode, a, y, mean, invstd, gamma, dgamma, dbeta, dy_out,
                 y2, mean2, invstd2, gamma2, dgamma2, dbeta2, dy2_out, dz_buf, gscale, accumulate)


def bn_bwd_finish(ws: "Workspace", part, G: int, nq: int, y, mean, invstd, gamma, dgamma, dbeta,
                  dz, dy_out, y2=None, mean2=None, invstd2=None, gamma2=None, dgamma2=None,
                  dbeta2=None, dy2_out=None, gscale: float = 1.0, accumulate: bool = False,
                  k_out: Optional[torch.Tensor] = None) -> None:
    """Finalize + apply of a BN backward whose reduction a dgrad epilogue already produced
    (partials ``part`` [G][nq][C], masked gradient ``dz``): ONE finalize launch (csrc/bn.hip
    bn_stats_kernel<1>: f64 slabs + last-arriver combine -> gamma/beta gradients and the apply
    coefficients of both branches), then the apply pass(es). SyncBatchNorm takes the separate
    reduce -> all-reduce -> finalize path.
    ``k_out`` (f32, 3 x C per branch: [k1; k2; k3] of branch 1, then of the shortcut branch; not
    SyncBatchNorm): the apply coefficients are written there and the apply pass of every branch
    whose output is None is skipped -- its consumer forms dy itself (:func:`conv_wgrad` ``bna``,
    :func:`conv_dgrad_bnf`)."""
    N, H, W, C_ = y.shape
    mode = 2 if nq == 3 else 1   # dz is materialised in both cases
    a = BwdArgs(None, None, None, 0, ptr(y), None, None, ptr(y2), None, None, mode, None, ptr(part),
                nq, N * H * W, C_)
    sync = getattr(ws, "sync_comm", None)
    if k_out is not None and ((sync is not None and sync.world_size > 1)
                              or k_out.numel() < 3 * (nq - 1) * C_):
        raise ValueError("bn_bwd_finish: k_out needs the non-synchronised form and 3 x C per branch")
    if sync is None or sync.world_size == 1:
        k = ws.get("bn_k", 6 * C_) if k_out is None else k_out
        S = _stats_slabs(G, C_)
        slabs = ws.get("bn_slabs", S * nq * C_, torch.float64)
        cnt = ws.counters(math.ceil(C_ / _stats_cg(C_)))
        o = ext.BnBwdOut(float(N * H * W), float(gscale), int(accumulate))
        o.gamma[0], o.mean[0], o.invstd[0] = ptr(gamma), ptr(mean), ptr(invstd)
        o.dgamma[0], o.dbeta[0] = ptr(dgamma), ptr(dbeta)
        if nq == 3:
            o.gamma[1], o.mean[1], o.invstd[1] = ptr(gamma2), ptr(mean2), ptr(invstd2)
            o.dgamma[1], o.dbeta[1] = ptr(dgamma2), ptr(dbeta2)
        o.k = ptr(k)
        L, st, dt = ext.lib(), stream(y.device), dt_of(y)
        check(L.pda_bn_bwd_stats(ptr(part), G, nq, C_, S, ptr(slabs), ptr(cnt), C.byref(o),
                                 _stats_cg(C_), st), "bn_bwd_stats")
        if mode == 2 and dy_out is not None and dy2_out is not None and _BWD_APPLY2 and \
                L.pda_bn_bwd_apply2(ptr(dz), ptr(y), ptr(y2), ptr(k), ptr(dy_out), ptr(dy2_out),
                                    N * H * W, C_, dt, st) == 0:
            return   # both branches in one pass over dz
        if dy_out is not None:
            check(L.pda_bn_bwd_apply(C.byref(a), ptr(dz), ptr(y), ptr(k[0:C_]), ptr(k[C_:2 * C_]),
                                     ptr(k[2 * C_:3 * C_]), ptr(dy_out), dt, st), "bn_bwd_apply")
        if mode == 2 and dy2_out is not None:
            check(L.pda_bn_bwd_apply(C.byref(a), ptr(dz), ptr(y2), ptr(k[3 * C_:4 * C_]),
                                     ptr(k[4 * C_:5 * C_]), ptr(k[5 * C_:6 * C_]), ptr(dy2_out), dt,
                                     st), "bn_bwd_apply2")
        return
    _bn_bwd_tail(ws, part, G, nq, mode, a, y, mean, invstd, gamma, dgamma, dbeta, dy_out,
                 y2, mean2, invstd2, gamma2, dgamma2, dbeta2, dy2_out, dz, gscale, accumulate)


# channels per block group of the statistics kernel (csrc/bn.hip stats_cg): a quad of channels gets
# 1024 / cg lanes, so narrower groups shorten both levels' serial load chains.  Measured in step
# (profiles/ab_r5.md section 17): 64-channel groups -0.12 ms/step against 256 since the round-5
# hand-off dropped its release fence (round 4, with the fence: 64 was +0.03), 32 -0.05; S =
# sqrt(0.75 T) slabs with at least 8 (0.2: +0.16, 1.5 / 3.0: within noise)
_BN_CG = 64
_BN_SK = 0.75
_BN_SMIN = 8


def _stats_cg(C_: int) -> int:
    return min(C_, _BN_CG)


def _stats_slabs(T: int, C_: int) -> int:
    """Blocks per channel group of the one-launch statistics kernel: level 1 reads T/S tiles per
    block, the group's last arriver S slabs -- S ~ sqrt(T) balances the two (both run at one CU's
    bandwidth), at least 8 when T allows so the level-1 reads spread over CUs."""
    return max(1, min(T, max(_BN_SMIN, int(math.sqrt(_BN_SK * T)))))


def _bn_bwd_tail(ws, part, G, nq, mode, a, y, mean, invstd, gamma, dgamma, dbeta, dy_out,
                 y2, mean2, invstd2, gamma2, dgamma2, dbeta2, dy2_out, dz_buf, gscale, accumulate):
    C_ = y.shape[-1]
    rows = y.numel() // C_
    st = stream(y.device)
    L = ext.lib()
    dt = dt_of(y)
    part, G = prereduce(part, G, nq * C_, ws)
    part, G, world = _sync_sums(part, G, nq * C_, ws)
    # SyncBN: the input-gradient coefficients need the GLOBAL sums, while gamma/beta keep the
    # per-rank gradient (torch SyncBatchNorm) that the DDP bucket average then combines
    gscale = gscale / world
    k = ws.get("bn_k", 6 * C_)
    check(L.pda_bn_bwd_finalize(ptr(part), G, nq, 1, C_, float(rows * world), ptr(gamma), ptr(mean),
                                ptr(invstd), ptr(dgamma), ptr(dbeta), ptr(k[0:C_]),
                                ptr(k[C_:2 * C_]), ptr(k[2 * C_:3 * C_]), float(gscale),
                                int(accumulate), st), "bn_bwd_finalize")
    if mode == 2:
        check(L.pda_bn_bwd_finalize(ptr(part), G, nq, 2, C_, float(rows * world), ptr(gamma2), ptr(mean2),
                                    ptr(invstd2), ptr(dgamma2), ptr(dbeta2), ptr(k[3 * C_:4 * C_]),
                                    ptr(k[4 * C_:5 * C_]), ptr(k[5 * C_:6 * C_]), float(gscale),
                                    int(accumulate), st), "bn_bwd_finalize2")
    dz_in = dz_buf if mode in (1, 2) else None
    check(L.pda_bn_bwd_apply(C.byref(a), ptr(dz_in), ptr(y), ptr(k[0:C_]), ptr(k[C_:2 * C_]),
                             ptr(k[2 * C_:3 * C_]), ptr(dy_out), dt, st), "bn_bwd_apply")
    if mode == 2:
        check(L.pda_bn_bwd_apply(C.byref(a), ptr(dz_buf), ptr(y2), ptr(k[3 * C_:4 * C_]),
                                 ptr(k[4 * C_:5 * C_]), ptr(k[5 * C_:6 * C_]), ptr(dy2_out), dt, st),
              "bn_bwd_apply2")


# ------------------------------------------------------------------ head / loss
def xent(logits: torch.Tensor, labels: torch.Tensor, loss_rows, loss, dlog=None,
         gscale: float = 1.0, gdev: Optional[torch.Tensor] = None) -> None:
    """loss_rows/loss (nullable) = CE(logits, labels); dlog (16-bit [B, ld]) = d(mean CE)/dlogits
    * gscale * gdev[0] (zero in the padding columns)."""
    B, K = logits.shape[0], logits.shape[1]
    ld_out = dlog.shape[1] if dlog is not None else 0
    dt = dt_of(dlog) if dlog is not None else 1
    rc = ext.lib().pda_xent(ptr(logits), B, K, logits.stride(0), ptr(labels), ptr(loss_rows), ptr(loss),
                            ptr(dlog), ld_out, float(gscale), ptr(gdev), dt, int(dlog is not None),
                            stream(logits.device))
    check(rc, "xent")


def topk_hits(logits, labels, hits) -> None:
    B, K = logits.shape
    rc = ext.lib().pda_topk(ptr(logits), B, K, logits.stride(0), ptr(labels), ptr(hits),
                            stream(logits.device))
    check(rc, "topk")


def col_sum(x, C_: int, out, scale: float = 1.0, accumulate: bool = False) -> None:
    rc = ext.lib().pda_col_sum(ptr(x), x.shape[0], C_, x.stride(0), float(scale), ptr(out), dt_of(x),
                               int(accumulate), stream(x.device))
    check(rc, "col_sum")


# ------------------------------------------------------------------ optimizer / amp
def sgd_flat(p, g, buf, shadow, lr, momentum, wd, initialized: bool, inv_scale=None,
             found_inf=None):
    """Fused SGD over the flat buffers; ``inv_scale`` / ``found_inf`` (device scalars published by
    :func:`amp_scan`) unscale the gradient and skip the whole update on overflow."""
    flags = (1 if initialized else 0) | (2 if shadow is not None else 0)
    dt = dt_of(shadow) if shadow is not None else 1
    rc = ext.lib().pda_sgd_flat(ptr(p), ptr(g), ptr(buf), ptr(shadow), p.numel(), float(lr),
                                float(momentum), float(wd), ptr(inv_scale), ptr(found_inf), flags, dt,
                                stream(p.device))
    check(rc, "sgd_flat")


def cast_flat(p, shadow) -> None:
    rc = ext.lib().pda_cast_flat(ptr(p), ptr(shadow), p.numel(), dt_of(shadow), stream(p.device))
    check(rc, "cast_flat")


def amp_scan(g, found_inf, inv_scale, scale, tracker, ws, growth=2.0, backoff=0.5,
             interval=2000) -> None:
    """One launch: found_inf = any non-finite in g; inv_scale = 1/scale; then (tracker given) the
    GradScaler update of scale/tracker -- all on the device, no host sync. ``ws``: int32[2] zeros
    (reset by the kernel itself)."""
    if g.numel() % 4 or g.dtype != torch.float32 or ws.dtype != torch.int32 or ws.numel() < 2:
        raise ValueError("amp_scan: f32 gradient with numel % 4 == 0 and an int32[2] workspace")
    check(ext.lib().pda_amp_scan(ptr(g), g.numel(), ptr(found_inf), ptr(inv_scale), ptr(scale),
                                 ptr(tracker), ptr(ws), float(growth), float(backoff), int(interval),
                                 stream(g.device)), "amp_scan")


def pack_stem(src_ohwi, dst, Cout=64, RS=49, Cin=3, Cpad=8) -> None:
    Kpad = dst.shape[1]
    check(ext.lib().pda_pack_stem(ptr(src_ohwi), ptr(dst), Cout, RS, Cin, Cpad, Kpad, dt_of(dst),
                                  stream(dst.device)), "pack_stem")


# ------------------------------------------------------------------ data
def synth_salt(seed: int, split: str) -> int:
    from ..data.synthetic import SPLIT_ID
    return ((seed * 97 + SPLIT_ID[split]) * 0x632BE5AB) & 0xFFFFFFFF


def synth_batch(ids: torch.Tensor, seed: int, split: str, num_classes: int, S: int, out, labels,
                keys) -> None:
    B = ids.numel()
    check(ext.lib().pda_synth(ptr(ids), B, synth_salt(seed, split), num_classes, ptr(keys),
                              ptr(labels), S, ptr(out), dt_of(out), stream(out.device)), "synth")


def nchw_to_nhwc8(x, out) -> None:
    B, C_, H, W = x.shape
    check(ext.lib().pda_nchw_to_nhwc8(ptr(x), B, C_, H, W, ptr(out), dt_of(out), stream(x.device)),
          "nchw_to_nhwc8")


# ------------------------------------------------------------------ stem (space-to-depth form)
def stem_s2d_geom(Nb: int, S: int) -> ConvGeom:
    """The 7x7/2/3 stem as a 4x4/1 conv with pad 2 on the 2x2 space-to-depth image (16 ch)."""
    return ConvGeom(Nb, S // 2, S // 2, 16, 64, 4, 4, 1, 2, ho=S // 2, wo=S // 2)


def synth_batch_s2d(ids, seed: int, split: str, num_classes: int, S: int, out, labels, keys) -> None:
    check(ext.lib().pda_synth_s2d(ptr(ids), ids.numel(), synth_salt(seed, split), num_classes,
                                  ptr(keys), ptr(labels), S, ptr(out), dt_of(out), stream(out.device)),
          "synth_s2d")


def nchw_to_s2d(x, out) -> None:
    B, C_, S, _ = x.shape
    check(ext.lib().pda_nchw_to_s2d(ptr(x), B, C_, S, ptr(out), dt_of(out), stream(x.device)),
          "nchw_to_s2d")


def pack_stem_s2d(src_ohwi, dst) -> None:
    check(ext.lib().pda_pack_stem_s2d(ptr(src_ohwi), ptr(dst), dst.shape[0], dt_of(dst),
                                      stream(dst.device)), "pack_stem_s2d")


def stem_s2d_grad(gpacked, grad_ohwi, accumulate: bool = False) -> None:
    check(ext.lib().pda_stem_s2d_grad(ptr(gpacked), ptr(grad_ohwi), gpacked.numel() // 256,
                                      int(accumulate), stream(gpacked.device)), "stem_s2d_grad")
