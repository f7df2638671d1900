"""pytorch_distributed_amd -- MI355X-native data-parallel ResNet training framework.

Same capabilities as HFAiLab/pytorch_distributed (single GPU, DataParallel,
DDP, mixed-precision DDP; checkpoint/resume on preemption), re-designed for
AMD Instinct MI355X (gfx950 / CDNA4): hand-written HIP kernels for the
ResNet hot path, a flat-buffer native training engine and RCCL over xGMI.
"""
__version__ = "0.1.0"

# (HIP-graph replay needs the runtime's single-queue graph launch, DEBUG_HIP_FORCE_GRAPH_QUEUES=1,
# set before HIP starts: the graph-replaying paths request it themselves and replay eagerly
# without it -- runtime/graphs.py request_single_queue_graphs; importing the package sets nothing)
from .config import RunConfig, config_for  # noqa: F401
