set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5j
timeout -k 10 400 python -u -m pytest tests/test_conv_shapes_gpu.py -k "halo" -x -q --timeout 200 --timeout-method thread > gpurun_out/r5j/tests.log 2>&1 || { tail -30 gpurun_out/r5j/tests.log; exit 1; }
tail -2 gpurun_out/r5j/tests.log
timeout -k 10 300 python tools/halo_bench.py 20 2>&1 | tee gpurun_out/r5j/halo.txt || exit 1
VARIANTS="- PDA_HALO_PRO=0 PDA_FUSE_PROLOGUE=1" REPS=2 TAG=r5j_ bash tools/gpu_ab_env.sh || exit 1
echo "== DEBUG_HIP_FORCE_GRAPH_QUEUES=0 --segments 1 --branches 1" | tee -a gpurun_out/r5j/repro.txt
DEBUG_HIP_FORCE_GRAPH_QUEUES=0 timeout -k 10 120 python tools/graph_queue_repro.py --segments 1 --branches 1 >> gpurun_out/r5j/repro.txt 2>&1
echo "rc=$?" | tee -a gpurun_out/r5j/repro.txt
