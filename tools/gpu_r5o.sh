set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5o
timeout -k 10 600 python -u -m pytest tests/test_native_model_gpu.py tests/test_production_shape_gpu.py tests/test_determinism_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5o/tests.log 2>&1 || { tail -30 gpurun_out/r5o/tests.log; exit 1; }
tail -2 gpurun_out/r5o/tests.log
VARIANTS="- PDA_TAIL_FUSE=nods" REPS=3 TAG=r5o_ bash tools/gpu_ab_env.sh
