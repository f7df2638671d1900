"""ResNet-50, single-process data parallel over all visible GPUs (reference: resnet_dp.py).

Global batch 3200 (= 400 per GPU on 8 GPUs), split across devices by
pytorch_distributed_amd.parallel.DataParallel. No CLI arguments needed; optional flags
mirror the MX_* env vars (``--help``).
"""
import os
import sys

# the DataParallel replicas replay HIP graphs: single-queue graph launch, set before HIP starts
# (pytorch_distributed_amd/runtime/graphs.py GRAPH_QUEUES_VAR)
os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "1")

from pytorch_distributed_amd.config import config_for  # noqa: E402
from pytorch_distributed_amd.trainer import run


def main():
    run(config_for("dp", argv=sys.argv[1:]), mode="dp")


if __name__ == "__main__":
    main()
