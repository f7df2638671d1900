set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5x
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "bn_" tests/test_production_shape_gpu.py tests/test_determinism_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5x/tests.log 2>&1 || { tail -30 gpurun_out/r5x/tests.log; exit 1; }
tail -2 gpurun_out/r5x/tests.log
KERNEL=bn_stats LIBS="- ab/libpda_kernels_bnold.so" bash tools/gpu_kernel_ab.sh || exit 1
VARIANTS="- PDA_KERNEL_LIB=ab/libpda_kernels_bnold.so" REPS=3 TAG=r5x_ bash tools/gpu_ab_env.sh
