"""ctypes bindings to ``_lib/libpda_kernels.so`` (the gfx950 HIP kernels).

The library exposes a C ABI of launchers that take raw device pointers and a
``hipStream_t``; no torch headers are compiled, so the build is fast and
ABI-independent of the PyTorch wheel. Every launcher returns the HIP error
code of the launch, which :func:`_check` turns into an exception -- ops never
fall back silently to PyTorch on a GPU box (a missing library raises).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path
from typing import Optional

import torch

__all__ = ["load", "available", "lib", "DT", "dt_of", "ConvDesc", "BwdArgs", "BnEpi", "BnFwdOut", "BnBwdOut",
           "stream", "ptr"]

_LIB: Optional[C.CDLL] = None
_ERR: Optional[str] = None
LIBPATH = Path(__file__).resolve().parent.parent / "_lib" / "libpda_kernels.so"
if os.environ.get("PDA_KERNEL_LIB"):   # A/B variants (tools/build_variant.py), relative to _lib/
    LIBPATH = LIBPATH.parent / os.environ["PDA_KERNEL_LIB"]

DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def dt_of(t) -> int:
    return DT[t if isinstance(t, torch.dtype) else t.dtype]


class ConvDesc(C.Structure):
    _fields_ = [(n, C.c_int) for n in
                ("Nb", "H", "W", "Cin", "Cout", "R", "S", "stride", "pad", "Ho", "Wo")]


class BwdArgs(C.Structure):
    _fields_ = [("g1", C.c_void_p), ("g2", C.c_void_p), ("gp", C.c_void_p), ("HW", C.c_int),
                ("y", C.c_void_p), ("sc", C.c_void_p), ("sh", C.c_void_p),
                ("y2", C.c_void_p), ("sc2", C.c_void_p), ("sh2", C.c_void_p),
                ("mode", C.c_int), ("dz_out", C.c_void_p),
                ("part", C.c_void_p), ("nq", C.c_int), ("rows", C.c_longlong), ("C", C.c_int)]


class BnEpi(C.Structure):
    """dgrad epilogue = BatchNorm-backward reduction (csrc/conv_gemm.hip ConvParams e*)."""
    _fields_ = [("mode", C.c_int), ("nq", C.c_int),
                ("y", C.c_void_p), ("sc", C.c_void_p), ("sh", C.c_void_p),
                ("y2", C.c_void_p), ("sc2", C.c_void_p), ("sh2", C.c_void_p),
                ("g2", C.c_void_p), ("part", C.c_void_p), ("mask", C.c_void_p)]


class BnFwdOut(C.Structure):
    """Outputs of the one-launch BatchNorm forward statistics (csrc/bn.hip bn_fwd_stats)."""
    _fields_ = [("gamma", C.c_void_p), ("beta", C.c_void_p),
                ("eps", C.c_float), ("momentum", C.c_float),
                ("mean", C.c_void_p), ("invstd", C.c_void_p), ("scale", C.c_void_p),
                ("shift", C.c_void_p), ("rmean", C.c_void_p), ("rvar", C.c_void_p),
                ("nbt", C.c_void_p), ("update", C.c_int), ("tot", C.c_void_p)]


class BnBwdOut(C.Structure):
    """Outputs of the one-launch BatchNorm backward finalize (csrc/bn.hip bn_stats_kernel<1>):
    branch 0 = the BN of y, branch 1 = the shortcut BN of y2; k = [branches][3][C]."""
    _fields_ = [("count", C.c_float), ("gscale", C.c_float), ("accumulate", C.c_int),
                ("gamma", C.c_void_p * 2), ("mean", C.c_void_p * 2), ("invstd", C.c_void_p * 2),
                ("dgamma", C.c_void_p * 2), ("dbeta", C.c_void_p * 2), ("k", C.c_void_p)]


class RedDescC(C.Structure):
    """One split-K reduction of pda_wgrad_reduce_batch (csrc/conv_gemm.hip RedDescC)."""
    _fields_ = [("slab", C.c_void_p), ("grad", C.c_void_p), ("ck", C.c_void_p), ("cB", C.c_void_p),
                ("cs", C.c_void_p)] + [(n, C.c_int) for n in
                                       ("splits", "M", "N", "cin_log2", "cin_real", "pitch",
                                        "accumulate")] + [("scale", C.c_float)]


_V, _I, _F, _L, _U, _D = C.c_void_p, C.c_int, C.c_float, C.c_longlong, C.c_uint, C.c_double
_SIGS = {
    "pda_conv_fwd": [C.POINTER(ConvDesc), _V, _V, _I, _V, _I, _I, _V, _V, _I, _V, _V, _I, _I, _I, _V],
    "pda_conv_fwd_tail": [C.POINTER(ConvDesc), _V, _V, _I, _V, _V, _V, _V, _V, _V, _V, _V, _V, _I, _I,
                          _I, _I, _V],
    "pda_conv_dgrad": [C.POINTER(ConvDesc), _V, _V, _V, C.POINTER(BnEpi), _I, _I, _I, _V],
    "pda_conv_dgrad_bnf": [C.POINTER(ConvDesc), _V, _V, _V, C.POINTER(BnEpi), _V, _V, _V, _V, _I, _I,
                           _I, _V],
    "pda_bn_fold": [_V, _V, _I, _I, _V, _V, _I, _V],
    "pda_wgrad_tap": [_V, _V, _V, _V, _V, _I, _I, _I, _I, _I, _I, _I, _I, _V],
    "pda_wgrad_stem_tap": [_V, _V, _V, _V, _V, _I, _I, _I, _I, _I, _I, _V],
    "pda_stem_fwd": [_V, _V, _V, _V, _I, _I, _I, _I, _I, _V],
    "pda_conv_wgrad": [C.POINTER(ConvDesc), _V, _V, _V, _I, _I, _V, _V, _I, _I, _I, _V],
    "pda_conv_wgrad_bna": [C.POINTER(ConvDesc), _V, _V, _V, _V, _V, _V, _V, _I, _I, _V, _V, _I, _I, _I,
                           _V],
    "pda_wgrad_reduce": [_V, _V, _I, _I, _I, _I, _I, _I, _F, _I, _V, _V, _V, _V],
    "pda_wgrad_reduce_batch": [C.POINTER(RedDescC), _I, _V],
    "pda_conv_wgrad_gram": [C.POINTER(ConvDesc), _V, _V, _V, _V, _I, _I, _I, _I, _I, _V],
    "pda_fold_bgemm": [_V, _V, _I, _I, _V, _I, _V],
    "pda_bn_fwd_stats": [_V, _I, _I, _I, _I, _I, _V, _V, C.POINTER(BnFwdOut), _I, _V],
    "pda_bn_bwd_stats": [_V, _I, _I, _I, _I, _V, _V, C.POINTER(BnBwdOut), _I, _V],
    "pda_bn_finalize_tot": [_V, _I, _D, _V, _V, _F, _F, _V, _V, _V, _V, _V, _V, _V, _I, _V],
    "pda_slab_reduce": [_V, _I, _I, _I, _V, _V],
    "pda_bn_eval_coeffs": [_V, _V, _V, _V, _F, _I, _V, _V, _V],
    "pda_bn_apply": [_V, _V, _V, _V, _V, _V, _V, _L, _I, _I, _I, _V, _I, _V],
    "pda_stem_pool": [_V, _V, _V, _V, _V, _I, _I, _I, _I, _I, _I, _I, _V],
    "pda_maxpool_bwd": [_V, _V, _V, _V, _I, _I, _I, _I, _I, _I, _I, _V],
    "pda_tail_pool": [_V, _V, _V, _V, _V, _V, _V, _I, _I, _I, _I, _I, _V],
    "pda_bn_bwd_reduce": [C.POINTER(BwdArgs), _I, _I, _V],
    "pda_stem_bwd_reduce": [_V, _V, _V, _V, _V, _V, _V, _V, _I, _I, _I, _I, _I, _I, _I, _I, _V],
    "pda_bn_bwd_finalize": [_V, _I, _I, _I, _I, _F, _V, _V, _V, _V, _V, _V, _V, _V, _F, _I, _V],
    "pda_bn_bwd_apply": [C.POINTER(BwdArgs), _V, _V, _V, _V, _V, _V, _I, _V],
    "pda_xent": [_V, _I, _I, _I, _V, _V, _V, _V, _I, _F, _V, _I, _I, _V],
    "pda_topk": [_V, _I, _I, _I, _V, _V, _V],
    "pda_col_sum": [_V, _I, _I, _I, _F, _V, _I, _I, _V],
    "pda_sgd_flat": [_V, _V, _V, _V, _L, _F, _F, _F, _V, _V, _I, _I, _V],
    "pda_cast_flat": [_V, _V, _L, _I, _V],
    "pda_amp_scan": [_V, _L, _V, _V, _V, _V, _V, _F, _F, _I, _V],
    "pda_pack_stem": [_V, _V, _I, _I, _I, _I, _I, _I, _V],
    "pda_synth": [_V, _I, _U, _I, _V, _V, _I, _V, _I, _V],
    "pda_nchw_to_nhwc8": [_V, _I, _I, _I, _I, _V, _I, _V],
    "pda_synth_s2d": [_V, _I, _U, _I, _V, _V, _I, _V, _I, _V],
    "pda_nchw_to_s2d": [_V, _I, _I, _I, _V, _I, _V],
    "pda_pack_stem_s2d": [_V, _V, _I, _I, _V],
    "pda_stem_s2d_grad": [_V, _V, _I, _I, _V],
    "pda_set_stream_cfg": [_I, _I, _I, _I],
    "pda_fork_probe": [_V, _V, _I, _V, _V],
    "pda_track": [_V, _V],
    "pda_track_count": [],
    "pda_event_create": [_V],
    "pda_event_create_flags": [_V, _U],
    "pda_event_record": [_V, _V],
    "pda_event_destroy": [_V],
    "pda_stream_wait_event": [_V, _V],
    "pda_bn_bwd_apply2": [_V, _V, _V, _V, _V, _V, _L, _I, _I, _V],
}


def stream_cfg() -> tuple:
    """16-bit BN apply passes (csrc/bn.hip StreamCfg): 4 chunks per thread + nontemporal loads /
    stores for tensors >= 50 MiB, the one-chunk kernels below, grid cap 65536 blocks. In-step A/B
    (tools/gpu_ab.sh, one box): 30.02 ms (one-chunk everywhere) vs 29.41 ms (100 MiB threshold);
    threshold 200 / 100 / 50 / 30 MiB: 29.38-29.53 / 29.16 / 29.06-29.11 / 29.02-29.13 ms; grid cap
    8192 / 16384 / 32768 / 65536: 29.53 / 29.15-29.27 / 28.90-29.09 / 28.86-28.97 ms."""
    # memory policy bits: 1 nontemporal loads, 2 nontemporal stores (write-through sc1 stores, bit
    # 4, measured +0.27 ms/step: profiles/ab_r4.md section 1)
    return (-1, 3, 65536, 50)


def load(required: bool = False) -> Optional[C.CDLL]:
    global _LIB, _ERR
    if _LIB is not None:
        return _LIB
    if not LIBPATH.exists() and os.environ.get("PDA_NO_BUILD") != "1":
        try:
            from .. import _build
            _build.build_kernels()
        except Exception as e:  # pragma: no cover
            _ERR = f"build failed: {e}"
    try:
        lib = C.CDLL(str(LIBPATH))
        for name, argt in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:   # an older A/B variant library (tools/build_variant.py)
                continue
            fn.argtypes = argt
            fn.restype = C.c_int
        if getattr(lib, "pda_set_stream_cfg", None) is not None:
            lib.pda_set_stream_cfg(*stream_cfg())
        _LIB = lib
    except OSError as e:
        _ERR = str(e)
        if required:
            raise RuntimeError(f"native kernels unavailable: {_ERR}") from e
    return _LIB


def available() -> bool:
    return load() is not None


def lib() -> C.CDLL:
    l = load(required=True)
    assert l is not None
    return l


def stream(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with HIP error {rc}")
