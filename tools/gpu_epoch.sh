#!/bin/bash
# GPU-box script: one FULL ImageNet-sized epoch (1,281,167 synthetic train samples + 50,000 val)
# through the reference entrypoint, i.e. the reference's own headline metric ("elapsed time per
# epoch", result.png), bs 400/GPU. DTYPES="bf16 fp32" selects the precisions.
set -o pipefail
mkdir -p gpurun_out/epoch
export PYTHONUNBUFFERED=1
for d in ${DTYPES:-bf16}; do
  rm -rf /tmp/epoch_run_$d   # checkpoints stay off gpurun_out/ (size cap on the copy-back)
  MX_EPOCHS=1 MX_DTYPE=$d MX_METRICS=1 MX_SAVE_PATH=/tmp/epoch_run_$d MX_LOG_EVERY=400 \
    timeout -k 10 ${EPOCH_TIMEOUT:-900} python resnet_single_gpu.py > gpurun_out/epoch/$d.log 2>&1 \
    || { echo "FAIL $d"; tail -20 gpurun_out/epoch/$d.log; exit 1; }
  cp /tmp/epoch_run_$d/metrics.jsonl gpurun_out/epoch/metrics_$d.jsonl
  echo "== $d"; grep -E "Epoch:|cost time|New Best" gpurun_out/epoch/$d.log
done
