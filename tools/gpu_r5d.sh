set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5d
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad_tap" tests/test_dp_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5d/tests.log 2>&1 || { tail -40 gpurun_out/r5d/tests.log; exit 1; }
tail -3 gpurun_out/r5d/tests.log
timeout -k 10 300 python -u tools/wgrad_tap_bench.py 2>&1 | tee gpurun_out/r5d/bench.txt
VARIANTS="PDA_WGRAD_TAP=56,28 PDA_WGRAD_TAP=0" REPS=2 TAG=r5d_ bash tools/gpu_ab_env.sh || exit 1
for q in 1 0; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 120 python -u tools/graph_queue_repro.py --side --segments 8 --iters 300 > gpurun_out/r5d/repro_q$q.txt 2>&1; echo "repro queues=$q rc=$?"; tail -2 gpurun_out/r5d/repro_q$q.txt
done
