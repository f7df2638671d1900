"""Native MI355X ResNet engine (placeholder until the HIP kernels land)."""
import torch


def supports(arch: str, dtype: torch.dtype) -> bool:
    return False
