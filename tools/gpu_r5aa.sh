set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5ac
timeout -k 10 300 python -u -m pytest tests/test_native_model_gpu.py -k "fork_tracking" -x -q --timeout 200 --timeout-method thread > gpurun_out/r5ac/tests.log 2>&1 || { tail -30 gpurun_out/r5ac/tests.log; exit 1; }
tail -2 gpurun_out/r5ac/tests.log
VARIANTS="- HIP_FORCE_DEV_KERNARG=1" REPS=4 TAG=r5ac_ bash tools/gpu_ab_env.sh
