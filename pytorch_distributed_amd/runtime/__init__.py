"""Runtime pieces around the native engine: HIP-graph capture of the training step."""
from .graphs import GraphedNativeStep, native_train_step

__all__ = ["GraphedNativeStep", "native_train_step"]
