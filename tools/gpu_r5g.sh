set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5g
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_shape_gpu.py tests/test_determinism_gpu.py tests/test_native_model_gpu.py tests/test_dp_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5g/tests.log 2>&1 || { tail -40 gpurun_out/r5g/tests.log; exit 1; }
tail -2 gpurun_out/r5g/tests.log
VARIANTS="- PDA_REDUCE_BATCH=0 PDA_WGRAD_TAP=0" REPS=2 TAG=r5g_ bash tools/gpu_ab_env.sh
