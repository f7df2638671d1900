set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5l
timeout -k 10 600 python -u -m pytest tests/test_conv_shapes_gpu.py tests/test_production_shape_gpu.py tests/test_native_model_gpu.py tests/test_determinism_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5l/tests.log 2>&1 || { tail -30 gpurun_out/r5l/tests.log; exit 1; }
tail -2 gpurun_out/r5l/tests.log
VARIANTS="- PDA_HALO64=0 PDA_HALO64=0,PDA_HALO_PRO=0" REPS=3 TAG=r5l_ bash tools/gpu_ab_env.sh || exit 1
for a in "--segments 1 --branches 0" "--segments 1 --branches 1"; do
  echo "== DEBUG_HIP_FORCE_GRAPH_QUEUES=0 $a" >> gpurun_out/r5l/repro.txt
  DEBUG_HIP_FORCE_GRAPH_QUEUES=0 timeout -k 10 120 python tools/graph_queue_repro.py $a >> gpurun_out/r5l/repro.txt 2>&1
  rc=$?; echo "rc=$rc" >> gpurun_out/r5l/repro.txt
  [ $rc -ne 0 ] && break
done
cat gpurun_out/r5l/repro.txt
