"""Native MI355X ResNet training engine (flat buffers + explicit forward/backward schedule).

What it replaces: the reference runs ``torchvision.models.resnet50()`` through
ATen/cuDNN/cuBLAS with autograd recording ~500 ops per step.
Here the whole network is ONE coarse autograd node whose forward and backward
are explicit schedules of our gfx950 kernels (``ops/native_ops.py``):

* activations are NHWC 16-bit (bf16 default, f16 for the AMP script); the input is
  generated/converted straight into the 2x2 space-to-depth layout (12 of 16 channels used),
  so the 7x7/2 stem becomes a 4x4/1 MFMA implicit GEMM with K = 256 (whole 16-B chunks);
* every conv is the implicit-GEMM MFMA kernel (fwd / dgrad / split-K wgrad); the
  forward epilogue emits BatchNorm partial statistics and its last-arriving
  workgroups finalize them inside the same launch, so BN costs one fused
  apply(+ReLU, +residual, +pool) pass (or nothing: the next conv's prologue);
* parameters live in ONE flat f32 buffer laid out in *gradient-production order*
  (fc, layer4.2 ... layer1.0, stem) so DDP buckets are contiguous slices that
  complete in order during backward; ``.grad`` of every parameter is a view into
  one flat f32 gradient buffer; a 16-bit shadow of the flat buffer (written by the
  fused SGD kernel) is what the convs read -- conv weights are stored OHWI
  (= ``torch.channels_last`` of the torchvision OIHW parameter), so the shadow
  needs no repacking (only the 9.4k-element stem is packed);
* BN running stats / counters live in flat buffers (one broadcast each for DDP).

The module keeps torchvision's module tree and ``state_dict`` keys: it adopts the
children of a :class:`~pytorch_distributed_amd.models.resnet.ResNet` instance and
re-points their parameters/buffers into the flat storage.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import math
import os
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple

import torch
from torch import nn

from ..ops import ext
from ..ops import native_ops as K
from ..ops.native_ops import ConvGeom, Workspace
from .resnet import Bottleneck, ResNet

__all__ = ["NativeResNet", "NativeSGD", "NativeCrossEntropy", "NativeTrainer", "supports"]

ALIGN = 64  # elements; keeps every segment 16-B aligned in the 16-bit shadow
# DDP bucket boundaries (block boundaries of the flat gradient) are padded to multiples of
# 8 ranks x 7 xGMI links x 256 B: every bucket then splits into equal 256-B-aligned per-rank /
# per-link slices for any world size dividing 8 (parallel/reducer.py cost model)
BUCKET_QUANTUM = 8 * 7 * 256 // 4   # f32 elements (3584)


def supports(arch: str, dtype: torch.dtype) -> bool:
    if dtype not in (torch.bfloat16, torch.float16, torch.float32):
        return False
    if arch not in ("resnet18", "resnet34", "resnet50", "resnet101", "resnet152"):
        return False
    return torch.cuda.is_available() and ext.available()


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def _align_q(n: int) -> int:
    return (n + BUCKET_QUANTUM - 1) // BUCKET_QUANTUM * BUCKET_QUANTUM


# ====================================================================== plan objects
@dataclass
class ConvBN:
    """One conv (+ the BatchNorm after it)."""
    name: str
    conv: nn.Conv2d
    bn: nn.BatchNorm2d
    cin_store: int            # channels of the stored input (stem: 16, space-to-depth)
    H: int                    # input spatial size
    W: int
    w_off: int = 0            # flat offsets
    w_len: int = 0
    bn_off: int = 0
    buf_off: int = 0
    nbt_idx: int = 0
    # per-step state (f32 [C] each): mean, invstd, scale, shift
    state: Optional[torch.Tensor] = None

    @property
    def cout(self) -> int:
        return self.conv.out_channels

    def geom(self, Nb: int) -> ConvGeom:
        c = self.conv
        if self.name == "stem":   # 7x7/2 on RGB == 4x4/1 on the 2x2 space-to-depth image
            return K.stem_s2d_geom(Nb, 2 * self.H)
        return ConvGeom(Nb, self.H, self.W, self.cin_store, c.out_channels, c.kernel_size[0],
                        c.kernel_size[1], c.stride[0], c.padding[0])

    @property
    def Ho(self) -> int:
        return self.geom(1).Ho


@dataclass
class Block:
    name: str
    units: List[ConvBN]               # main path; all but the last have ReLU
    ds: Optional[ConvBN]              # downsample conv+bn, or None (identity shortcut)
    seg: Tuple[int, int] = (0, 0)     # flat param range of this block


class NativeResNet(nn.Module):
    def __init__(self, ref: ResNet, device=None, dtype: torch.dtype = torch.bfloat16,
                 image_size: int = 224) -> None:
        super().__init__()
        device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("NativeResNet runs on the GPU; use the torch engine on CPU")
        ext.load(required=True)
        self.device = device
        self.dtype = dtype
        self.image_size = image_size
        self.num_classes = ref.fc.out_features
        self.arch_block = ref.block
        for name, child in ref.named_children():
            self.add_module(name, child)
        self.ws = Workspace(device)
        self._build_plan()
        self._allocate(ref)
        self._reducer = None
        self._grads_zero = True
        self._fwd_ctx = None
        self._anchor = torch.zeros((), device=device, requires_grad=True)
        # BN1/BN2 (+ReLU) applied inside the consumer conv's operand staging (fwd and wgrad):
        # "1" every consumer, "1x1" only 1x1 consumers (a 3x3 consumer gathers each element 9x per
        # N-tile, so it re-applies the prologue 9-36x: there one materialising pass is cheaper),
        # "1x1:H" also 3x3 consumers of input size >= H, "0" none
        # (round 4 re-check, "1x1" vs "1x1:56": within +-0.05 ms/step over two boxes -- kept,
        # profiles/ab_r4.md section 11)
        self.fuse_prologue = os.environ.get("PDA_FUSE_PROLOGUE", "1x1:56")
        self.fused_stem_bwd = True    # maxpool gather + ReLU mask + BN partials in one pass
        # the stem wgrad forms its dY from the BN backward in-kernel (WGRAD_BNA: no apply pass;
        # stem_bna = False keeps the apply-pass form for tests) and runs on the main stream, beside
        # layer1's weight gradients on the second stream (profiles/ab_r4.md section 8)
        self.stem_bna = True
        # PDA_STEM_SPLIT=1: the stem weight gradient in decomposed form, dW = k1 (dz^T X) +
        # k2 (y^T X) + k3 colsum(X) -- y^T X and the tap column sums of X run on the second stream
        # in the FORWARD (y0 and x0 are known there), so the backward's exposed tail reads dz and X
        # only (not dz and y); combined in the split-K reduce (eager world-1 steps; a DataParallel
        # capture and SyncBatchNorm keep WGRAD_BNA)
        self.stem_split = os.environ.get("PDA_STEM_SPLIT", "0") == "1"
        self.tail_mask = True         # tails store the ReLU bitmask the backward reads
        # a block's tail BN apply (+ residual + ReLU) runs inside the next block's conv1 forward,
        # which stages a = relu(bn3(y3) + r) from y3 and r and writes a once (FWD_TAIL); blocks whose
        # successor has a shortcut conv keep the apply pass (PDA_TAIL_FUSE=0: every tail does)
        self.tail_fuse = os.environ.get("PDA_TAIL_FUSE", "1") != "0"
        self.tail_fuse_ds = os.environ.get("PDA_TAIL_FUSE", "1") != "nods"
        # opt-in (PDA_REDUCE_BATCH=1): the second stream's split-K weight-gradient reductions
        # batched into one launch per stage (per block under DDP) instead of one per conv
        # (ops/native_ops.py ReduceBatch). Off by default: fewer launches and -79 us of kernel time,
        # but each stage's burst of reduce blocks slows the main chain's data-gradient convs beside it
        # (+0.25..0.4 ms/step in-step, profiles/ab_r5.md section 4)
        self.reduce_batching = os.environ.get("PDA_REDUCE_BATCH", "0") == "1"
        # consumer-side tail fold of the Bottleneck BN backward (see _block_backward)
        # ("0" off, "1" every stage, or the stages to fold, e.g. "12" = layer1 and layer2). Default
        # layer1-3: in-step A/B at the bench config (profiles/ab_r4.md) 28.26 ms off, 27.89 all
        # stages, 27.55 "12", 27.47 "123"; layer4's fold costs more than its apply pass (its G is
        # 512x512 over K = 2048 and its 7x7 dgrad has few tiles to hide the extra K). The
        # shortcut branch of a downsampling block keeps its apply pass and LDS-DMA weight-gradient
        # tile (folding it lost at every stage set, profiles/ab_r4.md section 5)
        fold = os.environ.get("PDA_BN_FOLD", "123")
        self.bn_fold = fold != "0"
        self.bn_fold_stages = None if fold in ("0", "1") else {int(c) for c in fold if c.isdigit()}
        # folded tails take conv3's weight gradient in the decomposed form diag(k1) dz^T a2 +
        # diag(k2) W3 Gram(a2) + k3 s^T: the Gram and column sums of a2 run in the forward on the
        # second stream, so the backward's GEMM is a plain dz^T a2 (no y3 read, no VALU transform)
        # (in-step A/B: 27.07 / 27.13 vs 27.22 / 27.20 ms/step, profiles/ab_r4.md section 8)
        self.bn_fold_wg = os.environ.get("PDA_BN_FOLD_WG", "1") != "0"
        self.ds_stream = True         # the shortcut conv runs on the second stream
        # weight gradients on a second HIP stream: nothing in the backward chain consumes them, so
        # the (compute-bound) wgrad GEMMs fill the CUs left idle by the (HBM-bound) BN-backward
        # passes and small finalize launches of the dgrad chain on the main stream
        self._side = (torch.cuda.Stream(device) if os.environ.get("PDA_WGRAD_STREAM", "1") != "0"
                      else None)
        self.ws_w = Workspace(device) if self._side is not None else self.ws
        # When the wgrad stream forks: "0" once per conv (eager default: each weight gradient
        # starts as soon as its inputs exist), "block" queues a residual block's weight-gradient
        # kernels and forks ONCE per block, "stage" once per stage (graph-capture default: in a
        # captured graph every fork / join edge becomes a cross-queue barrier packet); PDA_WGRAD_BATCH
        # overrides both (profiles/ab_r2_inlaunch_bn.md sections 9, 10)
        self._wbatch_env = os.environ.get("PDA_WGRAD_BATCH")
        # split-K block-target factor of this model's weight gradients (None: PDA_WGRAD_SCALE)
        self.wgrad_scale: Optional[float] = None
        self.set_wgrad_batch(self._wbatch_env or "0")
        self._keep: List[torch.Tensor] = []
        # called on the main stream with the flat-gradient offset below which every gradient is
        # final, after each residual block's backward (DataParallel splits its replica graphs there)
        self.segment_hook: Optional[Callable[[int], None]] = None
        # graph capture with the weight gradients in graphs of their own (parallel/dp.py
        # _ReplicaGraph side_split): the backward leaves the batched weight-gradient kernels queued
        # (no flush, no end-of-backward join) for the capture driver to record on the second stream
        self.defer_side = False
        # with defer_side: called right after each weight gradient is queued (its inputs are the
        # main-stream work issued so far), so a capture driver can end the main segment there
        self.wgrad_hook: Optional[Callable[[], None]] = None
        # fork tracking (csrc/common.h TRACKED_LAUNCH): while the native forward / backward runs
        # eagerly, every kernel launch on the main stream completes one event through its own
        # dispatch, and a fork to the second stream waits on that event instead of recording a
        # marker between kernels (the marker costs ~4-5 us of main-stream bubble per fork,
        # tools/fork_bench.py; ~60 forks per step). Off under graph capture, SyncBatchNorm (its
        # collectives run on the main stream) and PDA_FORK_TRACK=0.
        self.fork_tracking = os.environ.get("PDA_FORK_TRACK", "1") != "0"
        self._trk_ev = None
        self._trk_on = False
        # diagnostics (tools/layer_times.py): called on the main stream as probe(phase, name) after
        # the stem and after each residual block, forward and backward
        self.probe: Optional[Callable[[str, str], None]] = None
        self.refresh_shadow()

    def set_wgrad_batch(self, mode: str) -> None:
        """Wgrad-stream fork granularity ("0" | "block" | "stage", see __init__)."""
        if mode not in ("0", "block", "stage"):
            raise ValueError(f"PDA_WGRAD_BATCH={mode!r}: expected 0, block or stage")
        self._wbatch_mode = mode
        self._wbatch = [] if self._side is not None and mode != "0" else None

    @contextlib.contextmanager
    def graph_schedule(self, concurrent_side: bool = False):
        """Schedule for HIP-graph capture, for the duration of the block only: fork the wgrad
        stream once per stage (unless PDA_WGRAD_BATCH says otherwise): replayed 29.16-29.23 ms vs
        29.50-29.63 per block and 29.85-30.00 per conv (profiles/ab_r2_inlaunch_bn.md section 10).
        Eager steps before and after keep their schedule (the fork granularity changes no value:
        tests/test_graph_gpu.py checks the three modes bitwise). Refuses streams of non-default
        priority: hipStreamEndCapture segfaults on them (ROCm 7, profiles/ab_r3_dma.md §5)."""
        for st in (self._side,):
            if st is not None and st.priority != 0:
                raise RuntimeError("HIP graph capture of a non-default-priority stream crashes the "
                                   "HIP runtime at capture end; capture with default priorities")
        prev = self._wbatch_mode
        self.set_wgrad_batch(self._wbatch_env or "stage")
        # the HIP runtime replays a captured two-stream step almost serially
        # (profiles/rocprof_r3_graph_replay.md), so the weight gradients keep the per-kernel
        # split-K targets instead of the x0.7 of the concurrent eager step (DataParallel replay
        # 29.03 -> 28.85 ms/step, profiles/ab_r3_dma.md section 18). Per model: another model
        # running eagerly meanwhile keeps its own plans.
        prev_scale = self.wgrad_scale
        # (concurrent_side: the capture records the weight gradients as graphs of their own that
        # replay on the second stream beside the main chain, as the eager step runs them: they keep
        # the eager step's targets -- DataParallel replay 27.03-27.09 vs 27.12-27.24 ms at x1.0)
        if "PDA_WGRAD_SCALE" not in os.environ and not concurrent_side:
            self.wgrad_scale = 1.0
        try:
            yield
        finally:
            self.set_wgrad_batch(prev)
            self.wgrad_scale = prev_scale

    # ------------------------------------------------------------------ planning
    def _build_plan(self) -> None:
        S = self.image_size
        if S % 2:
            raise ValueError("image size must be even (space-to-depth stem)")
        self.stem = ConvBN("stem", self.conv1, self.bn1, 16, S // 2, S // 2)
        h = self.stem.Ho
        h = (h + 2 - 3) // 2 + 1  # maxpool 3x3/2/1
        self.pool_hw = h
        self.blocks: List[Block] = []
        for li in range(1, 5):
            layer = getattr(self, f"layer{li}")
            for bi, blk in enumerate(layer):
                nm = f"layer{li}.{bi}"
                cin = blk.conv1.in_channels
                units = []
                if isinstance(blk, Bottleneck):
                    u1 = ConvBN(nm + ".conv1", blk.conv1, blk.bn1, cin, h, h)
                    u2 = ConvBN(nm + ".conv2", blk.conv2, blk.bn2, blk.conv2.in_channels, h, h)
                    h2 = u2.Ho
                    u3 = ConvBN(nm + ".conv3", blk.conv3, blk.bn3, blk.conv3.in_channels, h2, h2)
                    units = [u1, u2, u3]
                else:
                    u1 = ConvBN(nm + ".conv1", blk.conv1, blk.bn1, cin, h, h)
                    h2 = u1.Ho
                    u2 = ConvBN(nm + ".conv2", blk.conv2, blk.bn2, blk.conv2.in_channels, h2, h2)
                    units = [u1, u2]
                ds = None
                if blk.downsample is not None:
                    ds = ConvBN(nm + ".downsample", blk.downsample[0], blk.downsample[1], cin, h, h)
                self.blocks.append(Block(nm, units, ds))
                h = units[-1].Ho
        self.final_hw = h
        self.feat_dim = self.fc.in_features
        if self.num_classes > 1024 or self.feat_dim % 64:
            raise ValueError("unsupported head shape")
        self.fc_rows = int(math.ceil(self.num_classes / 64) * 64)   # fc rows padded to the tile

    def _units_in_grad_order(self):
        """(block-or-None, [ConvBN...]) groups in backward completion order."""
        yield None, []  # fc (handled explicitly)
        for b in reversed(self.blocks):
            yield b, list(reversed(b.units)) + ([b.ds] if b.ds else [])
        yield "stem", [self.stem]

    def _allocate(self, ref: ResNet) -> None:
        dev = self.device
        off = 0
        # fc: bias then weight (padded rows)
        self.fc_b_off = off
        off += _align(self.num_classes)
        self.fc_w_off = off
        off += self.fc_rows * self.feat_dim
        off = _align_q(off)
        self.fc_seg_end = off
        self.block_bounds: List[int] = [off]
        units: List[ConvBN] = []
        for b, us in list(self._units_in_grad_order())[1:]:
            start = off
            for u in us:
                u.w_off = off
                u.w_len = u.conv.weight.numel()
                off += _align(u.w_len)
                u.bn_off = off
                off += 2 * _align(u.cout)   # gamma, beta
                units.append(u)
            off = _align_q(off)
            if isinstance(b, Block):
                b.seg = (start, off)
            self.block_bounds.append(off)
        self.numel = off
        self.units = units
        self.flat_params = torch.zeros(off, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(off, dtype=torch.float32, device=dev)
        # 16-bit engines: the convs read a 16-bit shadow of the f32 master weights (refreshed by the
        # fused SGD); the exact-fp32 engine reads the master weights themselves
        self.f32 = self.dtype == torch.float32
        self.flat_shadow = (self.flat_params if self.f32
                            else torch.zeros(off, dtype=self.dtype, device=dev))
        # BN buffers
        boff = 0
        for i, u in enumerate(units):
            u.buf_off = boff
            boff += 2 * _align(u.cout)
            u.nbt_idx = i
        # running mean/var (f32) and num_batches_tracked (int64) share ONE byte store, so DDP's
        # per-forward buffer sync (M4) is a single broadcast
        self.flat_bufstore = torch.zeros(boff * 4 + len(units) * 8, dtype=torch.uint8, device=dev)
        self.flat_buffers = self.flat_bufstore[:boff * 4].view(torch.float32)
        self.flat_nbt = self.flat_bufstore[boff * 4:].view(torch.int64)
        self.stem_packed = torch.zeros(64, 256, dtype=self.dtype, device=dev)   # [64][4][4][16]
        self.stem_wgrad = torch.zeros(64 * 256, dtype=torch.float32, device=dev)
        self._stem_k = torch.zeros(3 * 64, dtype=torch.float32, device=dev)   # fused stem BN-bwd
        self.bn_state = torch.zeros(sum(4 * _align(u.cout) for u in units), dtype=torch.float32,
                                    device=dev)
        so = 0
        for u in units:
            c = _align(u.cout)
            u.state = self.bn_state[so:so + 4 * c].view(4, c)[:, :u.cout]
            so += 4 * c
        # re-point parameters / buffers into the flat storage
        with torch.no_grad():
            for u in units:
                w = u.conv.weight
                O, I, R, S_ = w.shape
                seg = self.flat_params[u.w_off:u.w_off + u.w_len].view(O, R, S_, I)
                seg.copy_(w.detach().permute(0, 2, 3, 1))
                gseg = self.flat_grad[u.w_off:u.w_off + u.w_len].view(O, R, S_, I)
                self._rebind(u.conv, "weight", seg.permute(0, 3, 1, 2), gseg.permute(0, 3, 1, 2))
                c = u.cout
                ca = _align(c)
                for j, pn in enumerate(("weight", "bias")):
                    p = getattr(u.bn, pn)
                    s = self.flat_params[u.bn_off + j * ca:u.bn_off + j * ca + c]
                    s.copy_(p.detach())
                    self._rebind(u.bn, pn, s, self.flat_grad[u.bn_off + j * ca:u.bn_off + j * ca + c])
                rm = self.flat_buffers[u.buf_off:u.buf_off + c]
                rv = self.flat_buffers[u.buf_off + ca:u.buf_off + ca + c]
                rm.copy_(u.bn.running_mean)
                rv.copy_(u.bn.running_var)
                u.bn.running_mean = rm
                u.bn.running_var = rv
                nb = self.flat_nbt[u.nbt_idx:u.nbt_idx + 1].view(())
                nb.copy_(u.bn.num_batches_tracked)
                u.bn.num_batches_tracked = nb
            fw = self.flat_params[self.fc_w_off:self.fc_w_off + self.num_classes * self.feat_dim]
            fw = fw.view(self.num_classes, self.feat_dim)
            fw.copy_(self.fc.weight.detach())
            fgw = self.flat_grad[self.fc_w_off:self.fc_w_off + self.num_classes * self.feat_dim]
            self._rebind(self.fc, "weight", fw, fgw.view(self.num_classes, self.feat_dim))
            fb = self.flat_params[self.fc_b_off:self.fc_b_off + self.num_classes]
            fb.copy_(self.fc.bias.detach())
            self._rebind(self.fc, "bias", fb, self.flat_grad[self.fc_b_off:self.fc_b_off + self.num_classes])
        self.fc_w16 = self.flat_shadow[self.fc_w_off:self.fc_w_off + self.fc_rows * self.feat_dim].view(
            self.fc_rows, self.feat_dim)
        self.fc_wgrad_full = self.flat_grad[self.fc_w_off:self.fc_w_off + self.fc_rows * self.feat_dim]

    @staticmethod
    def _rebind(mod: nn.Module, name: str, data: torch.Tensor, grad: torch.Tensor) -> None:
        p = nn.Parameter(data, requires_grad=True)
        p.grad = grad
        mod._parameters[name] = p

    # ------------------------------------------------------------------ helpers
    def w16(self, u: ConvBN) -> torch.Tensor:
        if u is self.stem:
            return self.stem_packed
        O, I, R, S_ = u.conv.weight.shape
        return self.flat_shadow[u.w_off:u.w_off + u.w_len].view(O, R * S_ * I)

    def w16_ohwi(self, u: ConvBN) -> torch.Tensor:
        O, I, R, S_ = u.conv.weight.shape
        return self.flat_shadow[u.w_off:u.w_off + u.w_len].view(O, R, S_, I)

    def gamma(self, u):
        return self.flat_params[u.bn_off:u.bn_off + u.cout]

    def beta(self, u):
        ca = _align(u.cout)
        return self.flat_params[u.bn_off + ca:u.bn_off + ca + u.cout]

    def dgamma(self, u):
        return self.flat_grad[u.bn_off:u.bn_off + u.cout]

    def dbeta(self, u):
        ca = _align(u.cout)
        return self.flat_grad[u.bn_off + ca:u.bn_off + ca + u.cout]

    def rmean(self, u):
        return self.flat_buffers[u.buf_off:u.buf_off + u.cout]

    def rvar(self, u):
        ca = _align(u.cout)
        return self.flat_buffers[u.buf_off + ca:u.buf_off + ca + u.cout]

    def wgrad_view(self, u):
        return self.flat_grad[u.w_off:u.w_off + u.w_len]

    @torch.no_grad()
    def refresh_shadow(self) -> None:
        """16-bit shadow of the flat parameters (the SGD kernel keeps it fresh afterwards)."""
        if not self.f32:
            K.cast_flat(self.flat_params, self.flat_shadow)
        self._pack_stem()

    def _pack_stem(self) -> None:
        K.pack_stem_s2d(self.flat_params[self.stem.w_off:self.stem.w_off + self.stem.w_len],
                        self.stem_packed)

    def _empty(self, *shape, dtype=None) -> torch.Tensor:
        return torch.empty(*shape, dtype=self.dtype if dtype is None else dtype, device=self.device)

    # ------------------------------------------------------------------ DDP / DP hooks
    def grad_boundaries(self) -> List[int]:
        return list(self.block_bounds)

    def attach_reducer(self, reducer) -> None:
        self._reducer = reducer

    def stage_bounds(self) -> List[int]:
        """Flat-gradient offsets at which a stage's backward is complete (after layer4.0, layer3.0,
        layer2.0: the gradient below each offset is final), in backward order."""
        nblk = len(self.blocks)
        return [self.block_bounds[nblk - bi] for bi, b in enumerate(self.blocks)
                if bi > 0 and b.name.endswith(".0")][::-1]

    def join_side(self) -> None:
        """Make the current stream wait for everything queued on the weight-gradient stream
        (pending batched weight gradients are launched first)."""
        self._flush_wgrad()
        if self._side is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._side)

    @torch.no_grad()
    def set_sync_bn(self, comm) -> None:
        """SyncBatchNorm over ``comm`` (None: per-rank statistics, the reference's behaviour):
        every BN finalize of every workspace all-reduces its per-channel sums first."""
        for v in list(vars(self).values()):
            if isinstance(v, Workspace):
                v.sync_comm = comm

    def sync_from_rank0(self, comm) -> None:
        comm.broadcast(self.flat_params, 0)
        self.broadcast_buffers_from_rank0(comm)
        self.refresh_shadow()

    @torch.no_grad()
    def broadcast_buffers_from_rank0(self, comm, overlap: bool = False) -> None:
        """Running stats + counters from rank 0: ONE collective over the flat buffer store (DDP's
        per-forward buffer sync). ``overlap``: issued on the communicator's stream;
        the forward joins it right before the first BatchNorm finalize (the stem's), the first
        kernel that writes the store, so the batch generation and the stem conv run meanwhile."""
        if overlap:
            self._bufsync = (comm, comm.broadcast_async(self.flat_bufstore, 0))
            return
        comm.broadcast(self.flat_bufstore, 0)

    def _join_bufsync(self) -> None:
        pend = getattr(self, "_bufsync", None)
        if pend is not None:
            self._bufsync = None
            pend[0].wait(pend[1])

    def layout_signature(self) -> List[int]:
        """Integers every DDP rank must agree on before any collective (torch DDP's
        ``_verify_param_shape_across_processes``): flat sizes, geometry,
        precision and a digest of every parameter's shape and offset."""
        import zlib
        desc = ";".join(f"{n}:{tuple(p.shape)}:{(p.data_ptr() - self.flat_params.data_ptr()) // 4}"
                        for n, p in self.named_parameters())
        dt = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}[self.dtype]
        return [self.numel, self.flat_bufstore.numel(), self.image_size, dt, self.num_classes,
                len(self.block_bounds), zlib.crc32(desc.encode())]

    def zero_grad_flat(self) -> None:
        """The next backward OVERWRITES the flat gradient (its first write per segment does not
        accumulate), so no memset is issued: until then the ``.grad`` views keep the last values
        (torch 2.x's set_to_none leaves no gradient to read either)."""
        self._grads_zero = True

    # ------------------------------------------------------------------ input
    def input_generator(self, ds) -> Callable:
        """Loader hook: sample ids -> (model-ready input, int64 labels), generated on the device
        directly in the stem's 2x2 space-to-depth NHWC layout [B, S/2, S/2, 16] (16-bit)."""
        S = ds.image_size

        def gen(ids: torch.Tensor):
            if ids.device.type == "cpu" and not ids.is_pinned():
                # a pageable H2D copy blocks the host until the device has drained every earlier
                # launch (the whole previous step), after which the forward's small kernels run
                # ahead of the host's launches and leave the GPU idle between them (~0.7 ms/step
                # measured, tools/gap_analysis.py); from pinned memory the copy is a queued DMA
                ids = ids.pin_memory()
            ids_d = ids.to(self.device, non_blocking=True)
            B = ids_d.numel()
            x = self._empty(B, S // 2, S // 2, 16)
            lab = torch.empty(B, dtype=torch.int64, device=self.device)
            keys = torch.empty(B, dtype=torch.int32, device=self.device)
            K.synth_batch_s2d(ids_d, ds.seed, ds.split, ds.num_classes, S, x, lab, keys)
            return x, lab

        return gen

    def prepare_input(self, x: torch.Tensor) -> torch.Tensor:
        """Validate and convert the input BEFORE any kernel runs: every kernel's indexing assumes
        the plan's geometry, so a mismatched image size must never reach the GPU. Accepts NCHW
        images [B,3,S,S] (any float dtype) or the model-ready s2d layout [B,S/2,S/2,16]."""
        S = self.image_size
        if x.dtype == self.dtype and x.dim() == 4 and x.shape[-1] == 16:
            if tuple(x.shape[1:3]) != (S // 2, S // 2) or x.device != self.device:
                raise ValueError(f"s2d input {tuple(x.shape)} on {x.device} does not match the "
                                 f"planned {S}x{S} on {self.device}")
            return x.contiguous()
        if x.dim() != 4 or x.shape[1] != 3 or tuple(x.shape[2:]) != (S, S):
            raise ValueError(f"expected [B,3,{S},{S}] images or [B,{S // 2},{S // 2},16] "
                             f"{self.dtype} input, got {tuple(x.shape)}")
        xin = x.to(self.device, torch.float32).contiguous()
        out = self._empty(x.shape[0], S // 2, S // 2, 16)
        K.nchw_to_s2d(xin, out)
        return out

    # ------------------------------------------------------------------ forward
    def _fuse_into(self, u: ConvBN) -> bool:
        """Whether conv ``u`` applies the previous BN+ReLU in its operand staging (else the
        activation is materialised by bn_apply) -- the PDA_FUSE_PROLOGUE policy."""
        mode = self.fuse_prologue
        if mode in ("1", "0"):
            return mode == "1"
        if u.conv.kernel_size == (1, 1):
            return True
        return ":" in mode and u.H >= int(mode.split(":")[1])

    def _conv_bn(self, u: ConvBN, x: torch.Tensor, train: bool, pro=None, ws=None,
                 before_finalize=None, tail=None) -> torch.Tensor:
        """y = conv(x) and BN coefficients (batch stats in training, running stats in eval).
        ``pro=(scale, shift)``: x is the previous PRE-BN tensor; the conv applies BN+ReLU on load.
        ``tail`` (:class:`~..ops.native_ops.TailIn`): x is the previous block's pre-BN tail and the
        conv forms (and writes) that block's output while staging.
        ``before_finalize``: called between the conv launch and the BN finalize launch."""
        ws = self.ws if ws is None else ws
        Nb = x.shape[0]
        g = u.geom(Nb)
        y = self._empty(Nb, g.Ho, g.Wo, u.cout)
        st = u.state
        if train:   # batch statistics + BN finalize inside the conv launch
            bn = K.BnStats(ws, self.gamma(u), self.beta(u), u.bn.eps,
                           u.bn.momentum if u.bn.momentum is not None else 0.1,
                           st[0], st[1], st[2], st[3], self.rmean(u), self.rvar(u),
                           self.flat_nbt[u.nbt_idx:u.nbt_idx + 1], update_running=True)
            K.conv_fwd(x, self.w16(u), g, y, pro=pro, bn=bn, before_finalize=before_finalize,
                       tail=tail)
        else:
            K.conv_fwd(x, self.w16(u), g, y, pro=pro, tail=tail)
            if before_finalize is not None:
                before_finalize()
            K.bn_eval_coeffs(self.gamma(u), self.beta(u), self.rmean(u), self.rvar(u), u.bn.eps,
                             st[2], st[3])
        return y

    def _coeffs(self, u: ConvBN, train: bool):
        """(scale, shift) of unit ``u`` written by its finalize (train) / eval-coefficient kernel:
        views of the shared per-unit state, valid until the next forward of the same unit."""
        return u.state[2], u.state[3]

    def native_forward(self, x: torch.Tensor, train: bool, save: bool) -> torch.Tensor:
        self._track(train)
        try:
            return self._native_forward(x, train, save)
        finally:
            self._track(False)

    def _native_forward(self, x: torch.Tensor, train: bool, save: bool) -> torch.Tensor:
        x = self.prepare_input(x)
        Nb = x.shape[0]
        # per-unit BN state (mean/invstd/scale/shift) is referenced, not copied, by the saved
        # context; any later forward overwrites it, which the generation check in backward catches
        self._state_gen = getattr(self, "_state_gen", 0) + 1
        saved: Dict = {"x0": x, "gen": self._state_gen} if save else None
        # stem: conv -> bn -> relu -> maxpool (fused); a pending DDP buffer broadcast joins
        # before the stem's BN finalize (the first write of the running statistics)
        y0 = self._conv_bn(self.stem, x, train, before_finalize=self._join_bufsync)
        ph = self.pool_hw
        p = self._empty(Nb, ph, ph, self.stem.cout)
        arg = torch.empty(Nb, ph, ph, self.stem.cout, dtype=torch.uint8, device=self.device)
        sc, sh = self._coeffs(self.stem, train)
        K.stem_pool(y0, sc, sh, p, arg)
        if self.probe is not None:
            self.probe("fwd", "stem")
        gram_pending = False
        if save:
            saved["y0"], saved["arg"] = y0, arg
            saved["stem_stats"] = self.stem.state
            saved["blocks"] = []
            if self._stem_split_ok(Nb, y0):
                saved["stem_gram"] = self._stem_gram(x, y0)
                gram_pending = True
        h = p
        feat = None
        nblk = len(self.blocks)
        tail_in = None   # (y3, (sc, sh), TailIn): the previous tail, folded into this block's conv1
        for bi, b in enumerate(self.blocks):
            last = bi == nblk - 1
            rec = {"x": h} if save else None
            a = h
            ys, acts = [], [h]
            pro = None
            yd = None
            if tail_in is not None:
                a, pro = tail_in[0], tail_in[1]
            # (SyncBatchNorm: the shortcut BN's all-reduce must not run on a second stream beside
            # the main chain's -- two streams on one communicator can order its collectives
            # differently on different ranks and deadlock -- so the shortcut stays on the chain)
            ds_side = (b.ds is not None and self._side is not None and self.ds_stream
                       and self.ws.sync_comm is None)
            # with the previous tail folded into conv1, conv1 writes this block's input h: the
            # shortcut conv forks after it
            ds_late = ds_side and tail_in is not None
            cur = torch.cuda.current_stream(self.device)

            def fork_ds():   # the shortcut conv (+BN stats) beside conv1..conv3 on the 2nd stream
                self._fork()
                with torch.cuda.stream(self._side):
                    return self._conv_bn(b.ds, h, train, ws=self.ws_w)
            if ds_side and not ds_late:
                yd = fork_ds()
            gram_side = (save and train and self.bn_fold_wg and self._side is not None
                         and len(b.units) == 3 and self._tail_fold_ok(b, Nb))
            for j, u in enumerate(b.units):
                y = self._conv_bn(u, a, train, pro, tail=tail_in[2] if j == 0 and tail_in else None)
                if j == 0 and ds_late:
                    yd = fork_ds()
                ys.append(y)
                if save:
                    rec[f"s{j}"] = u.state
                if j < len(b.units) - 1:
                    sc, sh = self._coeffs(u, train)
                    if gram_side and j == len(b.units) - 2:
                        gB, gs, forked = self._fold_gram(b.units[-1], y, sc, sh)
                        rec["gram"] = (gB, gs)
                        gram_pending = gram_pending or forked
                    if self._fuse_into(b.units[j + 1]):
                        # the next conv applies BN+ReLU while staging its tiles
                        a, pro = y, (sc, sh)
                        acts.append(None)
                    else:
                        a, pro = self._empty(*y.shape), None
                        K.bn_apply(y, sc, sh, a, relu=True)
                        acts.append(a)
            if b.ds is not None:
                if ds_side:
                    cur.wait_stream(self._side)
                else:
                    yd = self._conv_bn(b.ds, h, train)
                if save:
                    rec["sd"] = b.ds.state
            ul = b.units[-1]
            sc, sh = self._coeffs(ul, train)
            tail_in = None
            nb = self.blocks[bi + 1] if not last else None
            # the tail's BN apply folds into the next block's conv1 (FWD_TAIL; a downsampling next
            # block forks its shortcut conv after that conv1); layers 1-2 only (conv1 of <= 128
            # channels, K <= 512): on the deep-K layers 3-4 the fused launch is slower than the
            # apply pass and the plain conv together (tools/tail_bench.py: layer1 422 vs 482 us,
            # layer2 233 vs 244, layer3 196 vs 142, layer4 214 vs 105 -- profiles/ab_r5.md
            # section 2). PDA_TAIL_FUSE=nods: not into downsampling blocks (the round-5 start)
            fuse = (nb is not None and self.tail_fuse and (nb.ds is None or self.tail_fuse_ds)
                    and nb.units[0].cout <= 128
                    and K.tail_fuse_ok(nb.units[0].geom(Nb), self.dtype))
            if last:
                feat = self._empty(Nb, ul.cout)
                if yd is not None:
                    K.tail_pool(ys[-1], sc, sh, feat, y2=yd, scale2=b.ds.state[2], shift2=b.ds.state[3])
                else:
                    K.tail_pool(ys[-1], sc, sh, feat, res=h)
                out = None
            else:
                out = self._empty(*ys[-1].shape)
                if yd is not None:
                    if fuse:
                        tail_in = (ys[-1], (sc, sh), K.TailIn(yd, out, sc2=b.ds.state[2],
                                                              sh2=b.ds.state[3]))
                    else:
                        K.bn_apply(ys[-1], sc, sh, out, y2=yd, scale2=b.ds.state[2],
                                   shift2=b.ds.state[3])
                else:
                    # identity tail: keep its ReLU bitmask (1/16 of the tensor) so the backward
                    # rebuilds the mask without re-reading the residual
                    mask = (torch.empty(out.numel() // 8, dtype=torch.uint8, device=self.device)
                            if save and self.tail_mask else None)
                    if fuse:
                        tail_in = (ys[-1], (sc, sh), K.TailIn(h, out, mask=mask))
                    else:
                        K.bn_apply(ys[-1], sc, sh, out, res=h, mask=mask)
                    if save:
                        rec["mask"] = mask
            if save:
                rec["ys"], rec["acts"], rec["yd"] = ys, acts, yd
                saved["blocks"].append(rec)
            h = out
            if self.probe is not None:
                self.probe("fwd", b.name)
        if gram_pending:
            # ONE join of the second stream's forward-time Gram work, after the last block: a join
            # per block stalled the main chain 20-55 us whenever a Gram was still running
            # (graph captures need every fork joined; the backward's weight gradients follow the
            # Grams on that stream anyway)
            torch.cuda.current_stream(self.device).wait_stream(self._side)
        logits = torch.empty(Nb, self.num_classes, dtype=torch.float32, device=self.device)
        g = ConvGeom(Nb, 1, 1, self.feat_dim, self.num_classes, 1, 1, 1, 0)
        K.conv_fwd(feat, self.fc_w16, g, logits, tile=self._fc_tile(),
                   bias=self.flat_params[self.fc_b_off:self.fc_b_off + self.num_classes])
        if save:
            saved["feat"] = feat
            saved["logits"] = logits
        self._fwd_ctx = saved
        return logits

    # ------------------------------------------------------------------ backward
    def _track(self, on: bool) -> None:
        """Arm / disarm fork tracking of this thread's launches on the current (main) stream."""
        L = ext.lib()
        if not on:
            if self._trk_on:
                L.pda_track(None, None)
                self._trk_on = False
            return
        if (not self.fork_tracking or self._side is None or self.defer_side
                or getattr(self.ws, "sync_comm", None) is not None
                or torch.cuda.is_current_stream_capturing()
                or getattr(L, "pda_track", None) is None):
            return
        if self._trk_ev is None:
            self._trk_ev = K.fork_event_create()
        L.pda_track(C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream), self._trk_ev)
        self._trk_on = True
        self._trk_c0 = L.pda_track_count()

    def __del__(self):
        ev = getattr(self, "_trk_ev", None)
        if ev is not None:
            try:
                ext.lib().pda_event_destroy(ev)
            except Exception:   # (interpreter shutdown: the library may be gone)
                pass

    def _fork(self) -> None:
        """The second stream waits for everything queued on the main stream so far: on the tracked
        event (completed by the latest native launch) when the main stream has issued a native
        launch since tracking was armed -- the forward / backward issue nothing else on it between
        forks -- else with a regular event record."""
        cur = torch.cuda.current_stream(self.device)
        L = ext.lib()
        if self._trk_on and L.pda_track_count() != self._trk_c0:
            K.check(L.pda_stream_wait_event(C.c_void_p(self._side.cuda_stream), self._trk_ev),
                    "pda_stream_wait_event")
        else:
            self._side.wait_stream(cur)

    def _wgrad(self, fn: Callable, *keep: torch.Tensor, split: bool = True) -> None:
        """Enqueue ``fn(workspace)`` (weight-gradient kernels) on the wgrad stream, ordered after
        everything queued so far on the main stream. Tensors the side stream reads are kept alive
        until the end-of-backward join, so the caching allocator cannot hand their memory to a
        main-stream allocation while the side stream may still be reading it. ``split=False``: the
        next weight gradient follows with no main-stream launch in between (a DataParallel capture
        records both in one side graph instead of ending an empty main segment)."""
        if self._side is None:
            fn(self.ws)
            return
        if self._wbatch is not None:
            self._wbatch.append(fn)
            self._keep.extend(keep)
            if split and self.defer_side and self.wgrad_hook is not None:
                self.wgrad_hook()   # (DataParallel capture: a side graph per weight gradient)
            return
        self._fork()
        with torch.cuda.stream(self._side):
            fn(self.ws_w)
        self._keep.extend(keep)

    def _flush_wgrad(self) -> None:
        """Run the queued weight-gradient kernels (PDA_WGRAD_BATCH=block) after one fork."""
        if not self._wbatch:
            return
        self._fork()
        with torch.cuda.stream(self._side):
            for fn in self._wbatch:
                fn(self.ws_w)
        self._wbatch.clear()

    def _flush_reduces(self) -> None:
        """Run the queued split-K reductions of the second stream's weight gradients (one launch)."""
        rb = self.ws_w.reduce_batch
        if rb is not None and rb.items:
            with torch.cuda.stream(self._side):
                rb.flush()

    def _grads_ready(self, red, upto: int) -> None:
        """DDP bucket readiness: the bucket's BN grads come from the main stream, its conv weight
        grads from the wgrad stream -- launch the all-reduce after both."""
        if self._side is None:
            red.grads_ready(upto)
            return
        self._flush_wgrad()
        self._flush_reduces()
        self._fork()
        with torch.cuda.stream(self._side):
            red.grads_ready(upto)

    def native_backward(self, dlog16: torch.Tensor) -> None:
        self._track(True)
        try:
            self._native_backward(dlog16)
        finally:
            self._track(False)

    def _native_backward(self, dlog16: torch.Tensor) -> None:
        """dlog16: [B, fc_rows] 16-bit d(loss)/d(logits) (zero padded).

        Schedule per bottleneck block (last to first): finish the tail BN backward (its reduction
        was fused into the NEXT block's conv1 dgrad epilogue) -> downsample wgrad/dgrad -> for
        conv3, conv2: wgrad + dgrad whose epilogue does the ReLU mask and the BN-backward partial
        sums of the preceding BN -> finish that BN -> conv1 wgrad + dgrad whose epilogue does the
        PREVIOUS block's tail reduction (adding the shortcut gradient). DDP buckets fire as each
        block's gradient segment completes."""
        sv = self._fwd_ctx
        if sv is None:
            raise RuntimeError("native backward without a saved forward")
        if sv["gen"] != self._state_gen:
            raise RuntimeError("another forward ran between this forward and its backward; the native "
                               "engine keeps one step of saved state (no retain_graph / interleaving)")
        acc = not self._grads_zero
        red = self._reducer
        if red is not None:
            red.reset()
        Nb = dlog16.shape[0]
        ws = self.ws
        # the second stream's split-K reductions are queued and run ONE launch per stage (per block
        # under DDP, whose buckets need each block's gradients) instead of one per weight gradient
        # (eager launches only: a graph capture records them where they are issued)
        self.ws_w.reduce_batch = (K.ReduceBatch(self.ws_w) if self.reduce_batching and
                                  self._side is not None and self._wbatch is None and
                                  not self.defer_side else None)
        # ---- fc
        gfc = ConvGeom(Nb, 1, 1, self.feat_dim, self.fc_rows, 1, 1, 1, 0)

        def fc_wgrad(w):
            K.col_sum(dlog16, self.num_classes,
                      self.flat_grad[self.fc_b_off:self.fc_b_off + self.num_classes], accumulate=acc)
            K.conv_wgrad(dlog16, sv["feat"], gfc, self.fc_wgrad_full, w, accumulate=acc,
                          wscale=self.wgrad_scale)
        self._wgrad(fc_wgrad, dlog16, sv["feat"])
        dfeat = self._empty(Nb, 1, 1, self.feat_dim)
        fc_w_ohwi = self.fc_w16.view(self.fc_rows, 1, 1, self.feat_dim)
        K.conv_dgrad(dlog16.view(Nb, 1, 1, self.fc_rows), fc_w_ohwi, gfc, dfeat, tile=self._fc_tile())
        if red is not None:
            self._grads_ready(red, self.block_bounds[0])
        # ---- last block's tail: standalone reduction of the pooled gradient
        nblk = len(self.blocks)
        b = self.blocks[-1]
        rec = sv["blocks"][-1]
        tail = self._tail_standalone(b, rec, dfeat.view(Nb, self.feat_dim), acc)
        shortcut_g = None
        for bi in range(nblk - 1, -1, -1):
            b = self.blocks[bi]
            rec = sv["blocks"][bi]
            prev = (self.blocks[bi - 1], sv["blocks"][bi - 1]) if bi > 0 else None
            dx_main, shortcut_g, tail = self._block_backward(b, rec, tail, prev, acc)
            if not self.defer_side and (self._wbatch_mode == "block" or b.ds is not None):
                self._flush_wgrad()
            if bi == 0 or self.blocks[bi - 1].name[:6] != b.name[:6]:
                self._flush_reduces()   # (stage boundary; under DDP _grads_ready flushes per block)
            if red is not None:
                self._grads_ready(red, self.block_bounds[nblk - bi])
            if self.segment_hook is not None:
                self.segment_hook(self.block_bounds[nblk - bi])
            if self.probe is not None:
                self.probe("bwd", b.name)
        # ---- stem: maxpool backward of (main + shortcut) gradients, BN backward, wgrad
        x0, y0, arg = sv["x0"], sv["y0"], sv["arg"]
        st0 = sv["stem_stats"]
        u = self.stem
        g0 = u.geom(Nb)
        sync = getattr(ws, "sync_comm", None)
        # the stem's BN-backward output feeds only its weight gradient: with the fused stem
        # backward, the wgrad forms dy0 = k1*dz0 + k2*y0 + k3 while staging (no apply pass, no
        # dy0 write + re-read: 2 x 642 MB at batch 400)
        bna = (self.fused_stem_bwd and self.stem_bna and (sync is None or sync.world_size == 1)
               and K.wgrad_bna_ok(g0, Nb, y0.dtype))
        if self.fused_stem_bwd:   # maxpool gather + ReLU mask + BN partials in one pass
            dz0 = self._empty(*y0.shape)
            part, G, nq = K.stem_bwd_reduce(ws, dx_main, arg, y0, st0[2], st0[3], dz0,
                                            dout2=shortcut_g)
            if bna:
                k0 = self._stem_k
                K.bn_bwd_finish(ws, part, G, nq, y0, st0[0], st0[1], self.gamma(u), self.dgamma(u),
                                self.dbeta(u), dz0, None, accumulate=acc, k_out=k0)
            else:
                dy0 = self._empty(*y0.shape)
                K.bn_bwd_finish(ws, part, G, nq, y0, st0[0], st0[1], self.gamma(u), self.dgamma(u),
                                self.dbeta(u), dz0, dy0, accumulate=acc)
        else:
            dy0 = self._empty(*y0.shape)
            dA0 = self._empty(*y0.shape)
            K.maxpool_bwd(dx_main, arg, dA0, dout2=shortcut_g)
            K.bn_bwd(ws, y0, st0[0], st0[1], self.gamma(u), st0[2], st0[3], self.dgamma(u),
                     self.dbeta(u), dy0, g1=dA0, accumulate=acc)
        if bna:
            sg = sv.get("stem_gram")

            def stem_wgrad(w):
                # (stem_s2d_grad reads the reduced gradient at once: its reduce runs unbatched)
                rb, w.reduce_batch = w.reduce_batch, None
                if sg is not None:   # decomposed: plain dz^T X, combined with k in the reduce
                    K.conv_wgrad(dz0, x0, g0, self.stem_wgrad, w, combine=(k0, sg[0], sg[1]),
                                 wscale=self.wgrad_scale)
                else:
                    K.conv_wgrad(dz0, x0, g0, self.stem_wgrad, w, bna=(y0, k0),
                                 wscale=self.wgrad_scale)
                w.reduce_batch = rb
                K.stem_s2d_grad(self.stem_wgrad, self.wgrad_view(u), accumulate=acc)
            if self._side is not None and not self.defer_side:
                # the main stream is idle after the stem's BN backward while the second stream still
                # drains layer1's weight gradients: the stem's runs beside them instead of after
                stem_wgrad(ws)
            else:
                self._wgrad(stem_wgrad, dz0, y0, x0, k0, split=False)   # (the last: no main work follows)
        else:
            def stem_wgrad(w):
                rb, w.reduce_batch = w.reduce_batch, None
                K.conv_wgrad(dy0, x0, g0, self.stem_wgrad, w, wscale=self.wgrad_scale)
                w.reduce_batch = rb
                K.stem_s2d_grad(self.stem_wgrad, self.wgrad_view(u), accumulate=acc)
            self._wgrad(stem_wgrad, dy0, x0, split=False)
        if not self.defer_side:
            self._flush_wgrad()
            self._flush_reduces()
            self.ws_w.reduce_batch = None
            if self._side is not None:   # join: the optimizer step reads every gradient
                torch.cuda.current_stream(self.device).wait_stream(self._side)
                self._keep.clear()
        if red is not None:
            red.grads_ready(self.block_bounds[-1])
            red.finish()
        self._grads_zero = False
        self._fwd_ctx = None

    def _tail_args(self, b: Block, rec, use_mask: bool = False):
        """Tensors describing a = relu(bn3(y3) + shortcut) of block b for the BN-backward."""
        ul = b.units[-1]
        sl = rec[f"s{len(b.units) - 1}"]
        d = dict(y=rec["ys"][-1], scale=sl[2], shift=sl[3])
        if b.ds is not None:
            sd = rec["sd"]
            d.update(y2=rec["yd"], scale2=sd[2], shift2=sd[3])
        elif use_mask and rec.get("mask") is not None:
            d.update(mask=rec["mask"])
        else:
            d.update(res=rec["x"])
        return d

    def _tail_standalone(self, b: Block, rec, gp, acc):
        """Tail reduction from the pooled head gradient (no producing dgrad to fuse into)."""
        ys = rec["ys"]
        dz = self._empty(*ys[-1].shape)
        ta = self._tail_args(b, rec)
        N, H, W, C_ = ys[-1].shape
        G = K._reduce_blocks(N * H * W, C_)
        nq = 3 if b.ds is not None else 2
        part = self.ws.get("bn_part", G * nq * C_)
        a = ext.BwdArgs(None, None, K.ptr(gp), H * W, K.ptr(ta["y"]), K.ptr(ta["scale"]),
                        K.ptr(ta["shift"]), K.ptr(ta.get("y2", ta.get("res"))), K.ptr(ta.get("scale2")),
                        K.ptr(ta.get("shift2")), 2 if b.ds is not None else 1, K.ptr(dz), K.ptr(part), nq,
                        N * H * W, C_)
        K.check(ext.lib().pda_bn_bwd_reduce(ext.C.byref(a), G, ext.dt_of(dz), ext.stream(dz.device)),
                "bn_bwd_reduce")
        return dz, part, G, nq

    def _tail_fold_ok(self, b: Block, Nb: int) -> bool:
        """Whether block ``b``'s tail BatchNorm backward is folded into its last conv (the
        consumer-side fold, PDA_BN_FOLD): 16-bit, a 1x1 last conv (Bottleneck conv3), per-rank
        statistics (SyncBatchNorm keeps the reduce / all-reduce / finalize path) and a weight-gradient
        plan the in-kernel BN operand (WGRAD_BNA) is built for."""
        ul = b.units[-1]
        if not self.bn_fold or self.f32 or ul.conv.kernel_size != (1, 1):
            return False
        if self.bn_fold_stages is not None and not (
                b.name.startswith("layer") and int(b.name[5]) in self.bn_fold_stages):
            return False
        sync = getattr(self.ws, "sync_comm", None)
        if sync is not None and sync.world_size > 1:
            return False
        g = ul.geom(Nb)
        return K.bnf_ok(g, self.dtype) and K.wgrad_bna_ok(g, Nb, self.dtype)

    def _fc_tile(self):
        """The head's fc GEMMs (M = batch rows, K = 2048): 64x64 tiles put twice the blocks of the
        default 64x128 on the chip -- 26.2 vs 33.0 us forward, 14.5 vs 17.1 us data gradient at
        batch 400 (tools/fc_probe.py, bit-identical logits). 16-bit only (the split-f32 engine has no
        double-buffered 64x64 tile)."""
        return (64, 64) if self.dtype in (torch.bfloat16, torch.float16) else None

    def _stem_split_ok(self, Nb: int, y0: torch.Tensor) -> bool:
        """Whether this training forward precomputes the stem weight gradient's y / colsum terms
        (``stem_split``): eager, a second stream, the fused WGRAD_BNA conditions."""
        sync = getattr(self.ws, "sync_comm", None)
        return (self.stem_split and self._side is not None and not self.defer_side
                and self.fused_stem_bwd and self.stem_bna and (sync is None or sync.world_size == 1)
                and y0.dtype in (torch.bfloat16, torch.float16)
                and K.wgrad_bna_ok(self.stem.geom(Nb), Nb, y0.dtype))

    def _stem_gram(self, x0: torch.Tensor, y0: torch.Tensor):
        """Forward-time terms of the decomposed stem weight gradient on the second stream:
        B = y0^T X (the stem's weight-gradient GEMM with dY := y0) and the per-tap column sums s
        of X; the forward joins the stream once after the last block."""
        g0 = self.stem.geom(x0.shape[0])
        self._fork()
        with torch.cuda.stream(self._side):
            B = torch.empty(g0.Cout * 16 * g0.Cin, dtype=torch.float32, device=self.device)
            K.conv_wgrad(y0, x0, g0, B, self.ws_w)
            s = K.stem_tap_colsum(x0, g0)
        return B, s

    def _fold_gram(self, ul: ConvBN, y2, sc, sh):
        """Forward-time half of the decomposed conv3 weight gradient, on the second stream beside
        conv3's forward: Gram(a2), the column sums s of a2 = relu(bn2(y2)), and B = W3 Gram(a2).
        Returns (B, s, forked): under a DataParallel capture with per-weight-gradient side graphs
        (``wgrad_hook``) the work is queued like a weight gradient and recorded as a side graph
        (forked = False: nothing for the forward to join)."""
        C_ = y2.shape[-1]
        if self.defer_side and self.wgrad_hook is not None and self._wbatch is not None:
            gram = torch.empty(C_ + 1, C_, dtype=torch.float32, device=self.device)
            B = torch.empty(ul.cout, C_, dtype=torch.float32, device=self.device)
            w16 = self.w16(ul)

            def fn(w, y2=y2, sc=sc, sh=sh, gram=gram, B=B, w16=w16):
                K.conv_wgrad_gram(y2, sc, sh, gram, w)
                K.fold_bgemm(w16, gram[:C_], B)
            self._wbatch.append(fn)
            self._keep.extend([y2, sc, sh, gram, B, w16])
            self.wgrad_hook()
            return B, gram[C_], False
        self._fork()
        with torch.cuda.stream(self._side):
            gram = torch.empty(C_ + 1, C_, dtype=torch.float32, device=self.device)
            K.conv_wgrad_gram(y2, sc, sh, gram, self.ws_w)   # Gram rows, then the column sums
            B = torch.empty(ul.cout, C_, dtype=torch.float32, device=self.device)
            K.fold_bgemm(self.w16(ul), gram[:C_], B)
        return B, gram[C_], True

    def _block_backward(self, b: Block, rec, tail, prev, acc):
        """Returns (dx_main, shortcut_grad, prev_tail) -- the last is the fused reduction of the
        previous block's tail, or None for the first block.

        Tail fold (Bottleneck blocks, PDA_BN_FOLD=1): the tail BN-backward output dy3 = k1*dz +
        k2*y3 + k3 is never materialised. Its two consumers take it from (dz, k): the conv3 weight
        gradient forms dy3 while staging (WGRAD_BNA), and the conv3 data gradient runs
        dX = dz . (k1 o W3) + a2 . G + W3^T k3 with G = W3^T diag(k2) W3 (y3 = a2 . W3^T is conv3's
        own forward; csrc/conv_gemm.hip DGRAD_BNF, bn_fold_kernel) -- the apply pass (read dz and
        y3, write dy3: three passes over the block's widest tensor) is gone from the chain."""
        ws = self.ws
        x = rec["x"]
        ys, acts, yd = rec["ys"], rec["acts"], rec["yd"]
        Nb = x.shape[0]
        n = len(b.units)
        ul = b.units[-1]
        sl = rec[f"s{n - 1}"]
        dz, part, G, nq = tail
        fold = self._tail_fold_ok(b, Nb)
        kt = (torch.empty((nq - 1) * 3 * ul.cout, dtype=torch.float32, device=self.device)
              if fold else None)
        dy = None if fold else self._empty(*ys[-1].shape)
        sc_ev = None
        if b.ds is not None:
            sd = rec["sd"]
            g = b.ds.geom(Nb)
            dyd = self._empty(*yd.shape)
            K.bn_bwd_finish(ws, part, G, nq, ys[-1], sl[0], sl[1], self.gamma(ul), self.dgamma(ul),
                            self.dbeta(ul), dz, dy, y2=yd, mean2=sd[0], invstd2=sd[1],
                            gamma2=self.gamma(b.ds), dgamma2=self.dgamma(b.ds), dbeta2=self.dbeta(b.ds),
                            dy2_out=dyd, accumulate=acc, k_out=kt)
            # shortcut branch first: its dX is the second gradient source of the previous tail.
            # On the second stream its dgrad overlaps the conv3/conv2 chain; an event marks it for
            # the conv1 dgrad epilogue (or the stem) that consumes it
            shortcut_g = self._empty(*x.shape)

            def ds_dgrad():
                K.conv_dgrad(dyd, self.w16_ohwi(b.ds), g, shortcut_g)
            if self._side is not None and self.ds_stream:
                self._fork()
                with torch.cuda.stream(self._side):
                    ds_dgrad()
                sc_ev = torch.cuda.Event()
                sc_ev.record(self._side)
                self._keep.extend([dz, x, kt, shortcut_g, dyd])
            else:
                ds_dgrad()
            self._wgrad(lambda w, u=b.ds, g=g, dyd=dyd: K.conv_wgrad(dyd, x, g, self.wgrad_view(u),
                                                                    w, accumulate=acc,
                                                                    wscale=self.wgrad_scale),
                        dyd, x, split=fold)   # (fold: bn_fold launches before conv3's wgrad)
        else:
            K.bn_bwd_finish(ws, part, G, nq, ys[-1], sl[0], sl[1], self.gamma(ul), self.dgamma(ul),
                            self.dbeta(ul), dz, dy, accumulate=acc, k_out=kt)
            shortcut_g = dz
        dx_main = None
        prev_tail = None
        cur = torch.cuda.current_stream(self.device)
        for j in range(n - 1, -1, -1):
            u = b.units[j]
            a_in = acts[j]
            g = u.geom(Nb)
            pro = None
            if a_in is None:   # fused prologue: recompute relu(bn(y_{j-1})) while staging B
                sp_ = rec[f"s{j - 1}"]
                a_in = ys[j - 1]
                pro = (sp_[2], sp_[3])
            bnf = None
            if fold and j == n - 1:
                # tail fold: (dz, k) stand for dy3 in both of conv3's gradients
                k3 = kt[:3 * u.cout]
                cin = u.conv.in_channels
                wf = self._empty(u.cout + cin, cin)
                fb = torch.empty(cin, dtype=torch.float32, device=self.device)
                K.bn_fold(self.w16(u), k3, wf, fb, ws)
                bnf = (wf, fb)
                if "gram" in rec:   # decomposed form: plain dz^T a2, combined in the split-K reduce
                    gB, gs = rec["gram"]
                    self._wgrad(lambda w, u=u, g=g, a=a_in, pro=pro, k3=k3, gB=gB, gs=gs:
                                K.conv_wgrad(dz, a, g, self.wgrad_view(u), w, accumulate=acc, pro=pro,
                                             combine=(k3, gB, gs), wscale=self.wgrad_scale),
                                dz, a_in, kt, gB, gs)
                else:
                    self._wgrad(lambda w, u=u, g=g, a=a_in, pro=pro, y3=ys[-1], k3=k3:
                                K.conv_wgrad(dz, a, g, self.wgrad_view(u), w, accumulate=acc, pro=pro,
                                             bna=(y3, k3), wscale=self.wgrad_scale),
                                dz, a_in, ys[-1], kt)
            else:
                self._wgrad(lambda w, u=u, g=g, dy=dy, a=a_in, pro=pro:
                            K.conv_wgrad(dy, a, g, self.wgrad_view(u), w, accumulate=acc, pro=pro,
                                         wscale=self.wgrad_scale), dy, a_in)

            def dgrad(out, epi=None, u=u, g=g, dy=dy, bnf=bnf, a_in=a_in, pro=pro):
                if bnf is not None:
                    K.conv_dgrad_bnf(dz, bnf[0], g, out, a_in, bnf[1], xa_pro=pro, epi=epi)
                else:
                    K.conv_dgrad(dy, self.w16_ohwi(u), g, out, epi=epi)
            out = self._empty(*a_in.shape)
            if j > 0:
                up = b.units[j - 1]
                sp = rec[f"s{j - 1}"]
                Gp = K.dgrad_slabs(g, Nb, dtype=ys[-1].dtype)
                # the dgrad's epilogue produces dz and the BN-backward partials of bn_{j-1}
                epi, part_p, nq_p = K.bn_epilogue(ws, Gp, ys[j - 1], sp[2], sp[3])
                dgrad(out, epi)                                      # out = dz of bn_{j-1}
                dyp = self._empty(*ys[j - 1].shape)
                K.bn_bwd_finish(ws, part_p, Gp, nq_p, ys[j - 1], sp[0], sp[1], self.gamma(up),
                                self.dgamma(up), self.dbeta(up), out, dyp, accumulate=acc)
                dy = dyp
            elif prev is not None:
                pb, prec = prev
                if sc_ev is not None:
                    cur.wait_event(sc_ev)
                Gp = K.dgrad_slabs(g, Nb, dtype=ys[-1].dtype)
                epi, part_p, nq_p = K.bn_epilogue(ws, Gp, g2=shortcut_g,
                                                  **self._tail_args(pb, prec, use_mask=True))
                dgrad(out, epi)                                      # out = dz of prev tail
                prev_tail = (out, part_p, Gp, nq_p)
            else:
                dgrad(out)
                dx_main = out
        if sc_ev is not None:   # the caller (next tail / stem backward) reads shortcut_g on main
            cur.wait_event(sc_ev)
        return dx_main, shortcut_g, prev_tail

    # ------------------------------------------------------------------ nn.Module API
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        train = self.training
        if train and torch.is_grad_enabled():
            return _NativeNetFn.apply(self._anchor, x, self)
        with torch.no_grad():
            return self.native_forward(x, train=train, save=False)

    def make_optimizer(self, lr=0.1, momentum=0.9, weight_decay=1e-4) -> "NativeSGD":
        return NativeSGD(self, lr=lr, momentum=momentum, weight_decay=weight_decay)

    def make_criterion(self) -> "NativeCrossEntropy":
        return NativeCrossEntropy(self)

    def _apply(self, fn, recurse=True):  # .to()/.cuda()/.half() would break the flat views
        return self

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        res = super().load_state_dict(state_dict, strict=strict)
        self.refresh_shadow()
        return res


class _NativeNetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, x, model: NativeResNet):
        ctx.model = model
        logits = model.native_forward(x, train=True, save=True)
        ctx.B = logits.shape[0]
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        m: NativeResNet = ctx.model
        pending = getattr(m, "_pending_dlog16", None)
        if pending is not None:
            dlog16 = pending
            m._pending_dlog16 = None
        else:  # generic criterion: convert f32 dlogits to the padded 16-bit buffer
            dlog16 = torch.zeros(ctx.B, m.fc_rows, dtype=m.dtype, device=m.device)
            dlog16[:, :m.num_classes].copy_(dlogits)
        m.native_backward(dlog16)
        return None, None, None   # the anchor only routes autograd here: no gradient, no fill


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, model: NativeResNet):
        B = logits.shape[0]
        loss_rows = torch.empty(B, dtype=torch.float32, device=logits.device)
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        K.xent(logits, labels, loss_rows, loss)
        ctx.save_for_backward(logits, labels)
        ctx.model = model
        return loss

    @staticmethod
    def backward(ctx, g):
        logits, labels = ctx.saved_tensors
        m: NativeResNet = ctx.model
        B = logits.shape[0]
        dlog16 = torch.empty(B, m.fc_rows, dtype=m.dtype, device=logits.device)
        gdev = g.reshape(1).to(torch.float32).contiguous()
        K.xent(logits, labels, torch.empty(B, device=logits.device), None, dlog=dlog16,
               gscale=1.0 / B, gdev=gdev)
        m._pending_dlog16 = dlog16
        # the dlogits handed to the network node are carried by dlog16; return a placeholder
        return torch.empty_like(logits), None, None


class NativeCrossEntropy(nn.Module):
    """CrossEntropyLoss (mean) fused with its gradient kernel for the native engine."""

    def __init__(self, model: Optional[NativeResNet] = None) -> None:
        super().__init__()
        self.model = model

    def forward(self, logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        m = self.model
        if m is None or not logits.is_cuda or logits.dtype != torch.float32:
            return nn.functional.cross_entropy(logits.float(), labels)
        if logits.requires_grad:
            return _XentFn.apply(logits, labels, m)
        B = logits.shape[0]
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        K.xent(logits.contiguous(), labels, torch.empty(B, device=logits.device), loss)
        return loss


class NativeSGD(torch.optim.Optimizer):
    """torch.optim.SGD semantics (momentum, dampening 0, weight decay on every parameter -- as the
    reference, quirk Q12) executed as ONE fused kernel over the flat buffers, which also refreshes
    the 16-bit weight shadow. ``state_dict()`` has torch SGD's format (per-parameter
    ``momentum_buffer``), so checkpoints interchange with the reference's optimizer."""

    def __init__(self, model: NativeResNet, lr=0.1, momentum=0.9, weight_decay=1e-4,
                 dampening=0.0, nesterov=False) -> None:
        if dampening != 0.0 or nesterov:
            raise ValueError("NativeSGD implements dampening=0, nesterov=False (reference settings)")
        defaults = dict(lr=lr, momentum=momentum, dampening=0.0, weight_decay=weight_decay,
                        nesterov=False, maximize=False, foreach=None, differentiable=False,
                        fused=None)
        super().__init__(list(model.parameters()), defaults)
        self.model = model
        self.flat_mom = torch.zeros_like(model.flat_params)
        self._initialized = False
        # per-parameter momentum views (torch format in state_dict)
        self._views = {}
        fp = model.flat_params
        base = fp.data_ptr()
        for p in self.param_groups[0]["params"]:
            off = (p.data_ptr() - base) // 4
            v = self.flat_mom[off:off + p.numel()]
            if p.dim() == 4:
                O, I, R, S_ = p.shape
                v = v.view(O, R, S_, I).permute(0, 3, 1, 2)
            else:
                v = v.view(p.shape)
            self._views[p] = v

    def zero_grad(self, set_to_none: bool = True) -> None:
        self.model.zero_grad_flat()

    def _launch_range(self, lo: int, hi: int, inv_scale=None, found_inf=None) -> None:
        g = self.param_groups[0]
        m = self.model
        K.sgd_flat(m.flat_params[lo:hi], m.flat_grad[lo:hi], self.flat_mom[lo:hi],
                   None if m.f32 else m.flat_shadow[lo:hi], g["lr"], g["momentum"],
                   g["weight_decay"], self._initialized, inv_scale=inv_scale, found_inf=found_inf)

    def _launch(self, inv_scale=None, found_inf=None) -> None:
        g = self.param_groups[0]
        m = self.model
        if m._grads_zero:
            # zero_grad() and no backward since: torch 2.x's set_to_none leaves every .grad None,
            # and SGD skips parameters without a gradient -- the flat gradient still holds the
            # previous step's values (no memset), so applying it would be a stale update
            return
        self._launch_range(0, m.numel, inv_scale, found_inf)
        m._pack_stem()
        # (an overflow-skipped first step leaves the momentum buffer unset on the device but the
        # flag set: the next step then reads the zero-initialised buffer, m*0 + d == d)
        self._initialized = True
        for p in g["params"]:
            self.state[p]["momentum_buffer"] = self._views[p]

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self._launch()
        return loss

    @torch.no_grad()
    def step_amp(self, scale: torch.Tensor, found_inf: torch.Tensor, tracker=None,
                 growth_factor: float = 2.0, backoff_factor: float = 0.5,
                 growth_interval: int = 2000) -> None:
        """AMP step, two launches and no host sync: ``amp_scan`` (non-finite check of the flat
        gradient; its last workgroup publishes found_inf and 1/scale and, given ``tracker``, runs
        the GradScaler scale update) then the fused SGD, which unscales by 1/scale and skips the
        whole update when found_inf is set."""
        if getattr(self, "_amp_ws", None) is None or self._amp_ws.device != scale.device:
            self._amp_ws = torch.zeros(2, dtype=torch.int32, device=scale.device)
            self._amp_inv = torch.ones(1, dtype=torch.float32, device=scale.device)
        K.amp_scan(self.model.flat_grad, found_inf, self._amp_inv, scale, tracker, self._amp_ws,
                   growth_factor, backoff_factor, growth_interval)
        self._launch(inv_scale=self._amp_inv, found_inf=found_inf)

    def state_dict(self):
        sd = super().state_dict()
        return sd

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        with torch.no_grad():
            any_buf = False
            for p in self.param_groups[0]["params"]:
                st = self.state.get(p, {})
                buf = st.get("momentum_buffer")
                if buf is not None:
                    self._views[p].copy_(buf)
                    st["momentum_buffer"] = self._views[p]
                    any_buf = True
            self._initialized = any_buf


# ====================================================================== bench trainer
class NativeTrainer:
    engine = "native"

    def __init__(self, arch, batch, dtype, device, world=1, rank=0, bucket_mb=32.0, image_size=224,
                 graph: bool = False):
        from .resnet import build_model
        from ..data.synthetic import SyntheticImageNet
        torch.manual_seed(0)
        ref = build_model(arch)
        self.model = NativeResNet(ref, device=device, dtype=dtype, image_size=image_size)
        self.net = self.model
        if world > 1:
            from ..parallel.ddp import DistributedDataParallel
            self.net = DistributedDataParallel(self.model, bucket_cap_mb=bucket_mb)
        self.opt = self.model.make_optimizer(lr=0.1, momentum=0.9, weight_decay=1e-4)
        self.crit = self.model.make_criterion()
        self.ds = SyntheticImageNet("train", seed=0, image_size=image_size)
        self.gen = self.model.input_generator(self.ds)
        self.batch, self.world, self.rank, self.device = batch, world, rank, device
        self.scaler = None
        if dtype == torch.float16:
            from ..amp import LossScaler
            self.scaler = LossScaler()
        self._loss = None
        self.graphed = None
        if graph:
            from ..runtime.graphs import graphs_unsafe_warning, single_queue_graphs
            if not single_queue_graphs():
                graphs_unsafe_warning("NativeTrainer(graph=True)")
                graph = False
        if graph:
            if world > 1:
                raise ValueError("graph capture of the distributed step is not enabled (RCCL "
                                 "collectives stay eager); use graph=False with world > 1")
            from ..runtime.graphs import GraphedNativeStep
            self.graphed = GraphedNativeStep(self.model, self.opt, self.gen, batch, self.scaler,
                                             device)

    def step(self, i: int) -> None:
        if self.graphed is not None:
            self.graphed.run((i * self.world + self.rank) * self.batch)
            self._loss = self.graphed.loss
            return
        ids = torch.arange(self.batch, dtype=torch.int64) + (i * self.world + self.rank) * self.batch
        x, y = self.gen(ids)
        out = self.net(x)
        loss = self.crit(out, y)
        if self.scaler is not None:
            self.scaler.scale(loss).backward()
            self.scaler.step(self.opt)
            self.scaler.update()
        else:
            loss.backward()
            self.opt.step()
        self.opt.zero_grad()
        self._loss = loss.detach()

    def last_loss(self):
        return None if self._loss is None else float(self._loss.item())

    def state_checksum(self) -> torch.Tensor:
        """Bit-exact checksum of master weights + momentum (bench cross-rank consistency)."""
        from ..bench_step import tensor_checksum
        return tensor_checksum([self.model.flat_params, self.opt.flat_mom])
