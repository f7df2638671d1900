#!/bin/bash
# GPU-box script: one FULL ImageNet-sized epoch (1,281,167 synthetic train samples + 50,000 val)
# through a reference entrypoint, i.e. the reference's own headline metric ("elapsed time per
# epoch", result.png, with its avg-GPU-util and GPU-memory panels from metrics.jsonl), bs 400/GPU.
# RUNS = space-separated <script>:<dtype> pairs; dtype "default" = the script's own precision
# (resnet_single_gpu.py fp32 as the reference, resnet_ddp_apex.py fp16 AMP).
set -o pipefail
mkdir -p gpurun_out/epoch
export PYTHONUNBUFFERED=1 PDA_NO_BUILD=1
for run in ${RUNS:-resnet_single_gpu.py:bf16}; do
  s=${run%%:*}; d=${run##*:}; tag=${s%.py}_$d
  rm -rf /tmp/epoch_run_$tag   # checkpoints stay off gpurun_out/ (size cap on the copy-back)
  dt=(); [ "$d" != default ] && dt=(MX_DTYPE=$d)
  env "${dt[@]}" MX_EPOCHS=1 MX_METRICS=1 MX_SAVE_PATH=/tmp/epoch_run_$tag MX_LOG_EVERY=400 \
    timeout -k 10 ${EPOCH_TIMEOUT:-900} python $s > gpurun_out/epoch/$tag.log 2>&1 \
    || { echo "FAIL $tag"; tail -20 gpurun_out/epoch/$tag.log; exit 1; }
  cp /tmp/epoch_run_$tag/metrics.jsonl gpurun_out/epoch/metrics_$tag.jsonl 2>/dev/null
  echo "== $tag"; grep -E "Epoch:|cost time|New Best" gpurun_out/epoch/$tag.log
  tail -2 gpurun_out/epoch/metrics_$tag.jsonl 2>/dev/null
done
