#!/bin/bash
# GPU-box script (round 3): per-stage step time (tools/layer_times.py, one and two streams), then
# the full-epoch panels of the fp32 single-GPU and fp16 AMP entrypoints (tools/gpu_epoch.sh).
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 240 python tools/layer_times.py --steps 10 > gpurun_out/layer_times_s1.txt 2>&1 || { tail -20 gpurun_out/layer_times_s1.txt; exit 1; }
timeout -k 10 240 python tools/layer_times.py --steps 10 --two-streams > gpurun_out/layer_times_s2.txt 2>&1 || { tail -20 gpurun_out/layer_times_s2.txt; exit 1; }
grep -v "^{" gpurun_out/layer_times_s1.txt | tail -12
RUNS="resnet_ddp_apex.py:default resnet_single_gpu.py:default" EPOCH_TIMEOUT=600 bash tools/gpu_epoch.sh
