#!/bin/bash
# GPU-box script: alternating in-step A/B of env settings (VARIANTS, REPS) -- a thin wrapper of
# gpu_ab_env.sh for one-line gpurun calls
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
VARIANTS="$V" REPS=${REPS:-3} TAG=${TAG:-q_} bash tools/gpu_ab_env.sh
