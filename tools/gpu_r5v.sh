set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
VARIANTS="- PDA_KERNEL_LIB=ab/libpda_kernels_convprio.so" REPS=3 TAG=r5w_ bash tools/gpu_ab_env.sh
