set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5m
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5m/tests.log 2>&1 || { tail -40 gpurun_out/r5m/tests.log; exit 1; }
tail -12 gpurun_out/r5m/tests.log
for a in "" "--side" "--side --threads 2" "--side --threads 4 --segments 8 --iters 500" "--threads 4 --segments 8 --branches 3 --iters 500"; do
  echo "== DEBUG_HIP_FORCE_GRAPH_QUEUES unset $a" >> gpurun_out/r5m/repro.txt
  env -u DEBUG_HIP_FORCE_GRAPH_QUEUES timeout -k 10 120 python tools/graph_queue_repro.py $a >> gpurun_out/r5m/repro.txt 2>&1
  rc=$?; echo "rc=$rc" >> gpurun_out/r5m/repro.txt
  [ $rc -ne 0 ] && break
done
cat gpurun_out/r5m/repro.txt
