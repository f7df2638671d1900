"""pytorch_distributed_amd -- MI355X-native data-parallel ResNet training framework.

Same capabilities as HFAiLab/pytorch_distributed (single GPU, DataParallel,
DDP, mixed-precision DDP; checkpoint/resume on preemption), re-designed for
AMD Instinct MI355X (gfx950 / CDNA4): hand-written HIP kernels for the
ResNet hot path, a flat-buffer native training engine and RCCL over xGMI.
"""
__version__ = "0.1.0"

from .config import RunConfig, config_for  # noqa: F401
