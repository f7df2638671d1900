#!/bin/bash
# GPU-box script (round 3 checkpoint): full GPU test suite, smoke, bench (all passes), then the
# fp16-AMP entrypoint's full epoch (after the comm-stream priority fix).
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
bash tools/gpu_check.sh || exit $?
RUNS="resnet_ddp_apex.py:default" EPOCH_TIMEOUT=400 bash tools/gpu_epoch.sh
