#!/bin/bash
# GPU-box script: per-step cost of each entrypoint's training loop at world 1 (MX_STEPS_PER_EPOCH
# steps + 1 validation step, "cost time per epoch" / steps), to find host-side overhead per config.
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1 MASTER_IP=127.0.0.1 MX_NPROCS=1
mkdir -p gpurun_out/entry
N=${STEPS:-300}
run() {  # tag script env...
  tag=$1; s=$2; shift 2
  env "$@" MX_EPOCHS=1 MX_STEPS_PER_EPOCH=$N MX_VAL_STEPS=1 MX_METRICS=1 MX_SAVE_PATH=/tmp/entry_$tag \
    timeout -k 10 300 python $s > gpurun_out/entry/$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 gpurun_out/entry/$tag.log; exit 1; }
  t=$(grep "cost time" gpurun_out/entry/$tag.log | awk '{print $5}')
  echo "$tag: $t s for $N steps -> $(python -c "print(round(1000*$t/$N,2))") ms/step"
}
run single_bf16 resnet_single_gpu.py MX_DTYPE=bf16 || exit 1
run single_fp16 resnet_single_gpu.py MX_DTYPE=fp16 || exit 1
run ddp_bf16 restnet_ddp.py MX_DTYPE=bf16 || exit 1
run apex_fp16 resnet_ddp_apex.py || exit 1
run apex_fp16_poll1000 resnet_ddp_apex.py MX_SUSPEND_POLL=1000 || exit 1
run apex_bf16 resnet_ddp_apex.py MX_DTYPE=bf16 || exit 1
