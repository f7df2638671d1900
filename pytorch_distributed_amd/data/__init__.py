from .sampler import DistributedSampler, SequentialIndices
from .synthetic import BatchLoader, SyntheticImageNet, synthetic_images, labels_for

__all__ = ["DistributedSampler", "SequentialIndices", "BatchLoader", "SyntheticImageNet",
           "synthetic_images", "labels_for"]
