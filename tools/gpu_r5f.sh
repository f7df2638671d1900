set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5f
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad_tap" -x -q --timeout 120 --timeout-method thread > gpurun_out/r5f/tests.log 2>&1 || { tail -40 gpurun_out/r5f/tests.log; exit 1; }
tail -2 gpurun_out/r5f/tests.log
timeout -k 10 300 python -u tools/wgrad_tap_bench.py 2>&1 | tee gpurun_out/r5f/bench.txt
