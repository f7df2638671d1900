"""pytorch_distributed_amd -- MI355X-native data-parallel ResNet training framework.

Same capabilities as HFAiLab/pytorch_distributed (single GPU, DataParallel,
DDP, mixed-precision DDP; checkpoint/resume on preemption), re-designed for
AMD Instinct MI355X (gfx950 / CDNA4): hand-written HIP kernels for the
ResNet hot path, a flat-buffer native training engine and RCCL over xGMI.
"""
__version__ = "0.1.0"

import os as _os

# HIP graphs replay on ONE hardware queue: the runtime's multi-queue graph launch (parallel branches
# spread over internal streams) segfaulted inside hipGraphLaunch (an out-of-range read of its
# stream list) in a long GPU test session -- tests/test_dp_gpu.py single-graph DataParallel
# capture after ~85 other tests; never with this setting. The captured step's branches already
# replayed almost serially (profiles/rocprof_r3_graph_replay.md); explicit two-stream concurrency
# is kept by replaying separate graphs on separate streams (PDA_DP_SIDE). Read by the HIP runtime
# at its initialisation: this import must come before the first HIP call (bench.py, the scripts
# and tests/conftest.py import the package first). Export the variable to override.
_os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "1")

from .config import RunConfig, config_for  # noqa: F401
