set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5k
timeout -k 10 400 python -u -m pytest tests/test_conv_shapes_gpu.py -k "halo" -x -q --timeout 200 --timeout-method thread > gpurun_out/r5k/tests.log 2>&1 || { tail -30 gpurun_out/r5k/tests.log; exit 1; }
tail -2 gpurun_out/r5k/tests.log
timeout -k 10 300 python tools/halo_bench.py 20 2>&1 | tee gpurun_out/r5k/halo.txt || exit 1
