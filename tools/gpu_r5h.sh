set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
KERNEL=bn_stats LIBS="- ab/libpda_kernels_bnu16.so ab/libpda_kernels_bnu8.so" bash tools/gpu_kernel_ab.sh || exit 1
VARIANTS="- PDA_KERNEL_LIB=ab/libpda_kernels_bnu16.so PDA_KERNEL_LIB=ab/libpda_kernels_bnu8.so" REPS=3 TAG=r5h_ bash tools/gpu_ab_env.sh
