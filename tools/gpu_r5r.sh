set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
VARIANTS="- PDA_WGRAD_BATCH=block" REPS=3 TAG=r5r_ bash tools/gpu_ab_env.sh
