"""ResNet-50 on one GPU (reference: resnet_single_gpu.py).

No CLI arguments needed; optional flags mirror the MX_* env vars (``--help``).

Overrides via MX_* env vars (see pytorch_distributed_amd/config.py), e.g.
``MX_EPOCHS=1 MX_STEPS_PER_EPOCH=50 python resnet_single_gpu.py``.
"""
import os
import sys

os.environ.setdefault("HIP_VISIBLE_DEVICES", os.environ.get("CUDA_VISIBLE_DEVICES", "0"))

from pytorch_distributed_amd.config import config_for  # noqa: E402
from pytorch_distributed_amd.trainer import run  # noqa: E402


def main():
    run(config_for("single", argv=sys.argv[1:]), mode="single")


if __name__ == "__main__":
    main()
