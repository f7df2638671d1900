#!/bin/bash
# GPU-box script (round 3, final tree): GPU test suite, smoke, bench (all passes), full epochs of the
# bf16 single-GPU and fp16 AMP entrypoints.
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
bash tools/gpu_check.sh || exit $?
RUNS="resnet_single_gpu.py:bf16 resnet_ddp_apex.py:default" EPOCH_TIMEOUT=400 bash tools/gpu_epoch.sh
