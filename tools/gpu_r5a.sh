set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5a
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "tail or fold" tests/test_dp_gpu.py tests/test_production_shape_gpu.py tests/test_determinism_gpu.py tests/test_native_model_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5a/tests.log 2>&1 || { tail -40 gpurun_out/r5a/tests.log; exit 1; }
tail -3 gpurun_out/r5a/tests.log
VARIANTS="PDA_TAIL_FUSE=1 PDA_TAIL_FUSE=0" REPS=3 TAG=r5a_ bash tools/gpu_ab_env.sh
