"""Run configuration: the reference's hard-coded hyper-parameters + env overrides.

The reference has no config system: every script hard-codes the same block in
``main()`` (reference ``resnet_single_gpu.py:70-78``, ``resnet_dp.py:67-75``,
``restnet_ddp.py:76-84``, ``resnet_ddp_apex.py:80-88``). :class:`RunConfig`
reproduces those defaults exactly per script; because the CLI takes no
arguments, overrides come from ``MX_*`` environment variables (additive: with
no env set, behaviour equals the reference).
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass
from typing import Optional, Sequence

__all__ = ["RunConfig", "SCRIPT_DEFAULTS", "config_for", "parse_cli"]


@dataclass(frozen=True)
class RunConfig:
    script: str = "single"           # single | dp | ddp | ddp_amp
    epochs: int = 100
    batch_size: int = 400            # per process (DP: global, see SCRIPT_DEFAULTS)
    num_workers: int = 4
    lr: float = 0.1
    momentum: float = 0.9
    weight_decay: float = 1e-4
    lr_step: int = 30
    lr_gamma: float = 0.1
    save_path: str = "output/resnet_single"
    arch: str = "resnet50"
    num_classes: int = 1000
    # --- framework extensions (MX_* env) ---
    dtype: str = "auto"              # auto | fp32 | bf16 | fp16 (auto: fp32 = the reference's precision; ddp_amp: fp16)
    device: str = "auto"             # auto | cuda | cpu
    data: str = "synthetic"          # synthetic | folder:<path>
    image_size: int = 224
    train_samples: int = 1_281_167   # ImageNet-1k train size (virtual synthetic samples)
    val_samples: int = 50_000
    steps_per_epoch: Optional[int] = None   # cap on train steps per epoch
    val_steps: Optional[int] = None         # cap on val steps per epoch
    empty_cache: str = "off"         # off | step | epoch  (reference: per-step for DP/DDP, quirk Q8)
    engine: str = "auto"             # auto | native | torch
    seed: int = 0
    log_every: int = 100
    metrics: bool = False            # write output/<run>/metrics.jsonl
    bucket_mb: float = 0.0           # DDP bucket cap (0 = framework default)
    sync_bn: bool = False            # SyncBatchNorm in DDP (reference: per-GPU statistics)
    graph: bool = False              # single-GPU native engine: replay each step from a HIP graph

    def replace(self, **kw) -> "RunConfig":
        return dataclasses.replace(self, **kw)


SCRIPT_DEFAULTS = {
    "single": dict(batch_size=400, save_path="output/resnet_single", empty_cache="epoch"),
    "dp": dict(batch_size=3200, save_path="output/resnet_dp", empty_cache="epoch"),
    "ddp": dict(batch_size=400, save_path="output/resnet_ddp"),
    "ddp_amp": dict(batch_size=400, save_path="output/resnet_ddp_amp", dtype="fp16"),
}

_ENV = {
    "MX_EPOCHS": ("epochs", int),
    "MX_BATCH": ("batch_size", int),
    "MX_WORKERS": ("num_workers", int),
    "MX_LR": ("lr", float),
    "MX_SAVE_PATH": ("save_path", str),
    "MX_ARCH": ("arch", str),
    "MX_NUM_CLASSES": ("num_classes", int),
    "MX_DTYPE": ("dtype", str),
    "MX_DEVICE": ("device", str),
    "MX_DATA": ("data", str),
    "MX_IMAGE_SIZE": ("image_size", int),
    "MX_TRAIN_SAMPLES": ("train_samples", int),
    "MX_VAL_SAMPLES": ("val_samples", int),
    "MX_STEPS_PER_EPOCH": ("steps_per_epoch", int),
    "MX_VAL_STEPS": ("val_steps", int),
    "MX_EMPTY_CACHE": ("empty_cache", str),
    "MX_ENGINE": ("engine", str),
    "MX_SEED": ("seed", int),
    "MX_LOG_EVERY": ("log_every", int),
    "MX_METRICS": ("metrics", lambda s: s not in ("", "0", "false", "False")),
    "MX_BUCKET_MB": ("bucket_mb", float),
    "MX_SYNC_BN": ("sync_bn", lambda s: s not in ("", "0", "false", "False")),
    "MX_GRAPH": ("graph", lambda s: s not in ("", "0", "false", "False")),
}


def _flag(var: str) -> str:
    return "--" + var[3:].lower().replace("_", "-")     # MX_STEPS_PER_EPOCH -> --steps-per-epoch


def parse_cli(argv: Sequence[str]) -> dict:
    """Optional command-line flags mirroring the ``MX_*`` variables (additive: the reference
    scripts take no arguments, and with none given nothing changes). Returns {env var: value}."""
    import argparse
    ap = argparse.ArgumentParser(add_help=True, description="MX_* overrides as flags")
    for var in _ENV:
        ap.add_argument(_flag(var), dest=var, default=None, metavar=var,
                        help=f"same as {var}")
    ns = ap.parse_args(list(argv))
    return {k: v for k, v in vars(ns).items() if v is not None}


def config_for(script: str, env: Optional[dict] = None,
               argv: Optional[Sequence[str]] = None) -> RunConfig:
    """Defaults of ``script`` (reference hyper-params) overlaid with ``MX_*`` env, then with the
    equivalent command-line flags (``argv``, e.g. ``--epochs 1 --steps-per-epoch 50``)."""
    if script not in SCRIPT_DEFAULTS:
        raise ValueError(f"unknown script {script!r}")
    env = dict(os.environ if env is None else env)
    if argv:
        env.update(parse_cli(argv))
    kw = dict(SCRIPT_DEFAULTS[script])
    kw["script"] = script
    for var, (name, conv) in _ENV.items():
        if var in env and env[var] != "":
            kw[name] = conv(env[var])
    cfg = RunConfig(**kw)
    if cfg.dtype not in ("auto", "fp32", "bf16", "fp16"):
        raise ValueError(f"MX_DTYPE must be auto|fp32|bf16|fp16, got {cfg.dtype!r}")
    if cfg.empty_cache not in ("off", "step", "epoch"):
        raise ValueError(f"MX_EMPTY_CACHE must be off|step|epoch, got {cfg.empty_cache!r}")
    return cfg
