set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5b
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "tail" -x -q --timeout 120 --timeout-method thread > gpurun_out/r5b/tests.log 2>&1 || { tail -40 gpurun_out/r5b/tests.log; exit 1; }
tail -2 gpurun_out/r5b/tests.log
timeout -k 10 300 python -u tools/tail_bench.py 2>&1 | tee gpurun_out/r5b/tail_bench.txt
VARIANTS="PDA_TAIL_FUSE=1 PDA_TAIL_FUSE=0" REPS=2 TAG=r5b_ bash tools/gpu_ab_env.sh
