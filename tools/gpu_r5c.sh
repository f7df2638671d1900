set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
VARIANTS="PDA_TAIL_FUSE=1 PDA_TAIL_FUSE=0" REPS=3 TAG=r5c_ bash tools/gpu_ab_env.sh
