set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dp_test.log 2>&1; rc=$?; tail -5 gpurun_out/dp_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/rccl_bench.py > gpurun_out/rccl_bench.txt 2> gpurun_out/rccl_bench.err || { tail -20 gpurun_out/rccl_bench.err; exit 1; }
tail -3 gpurun_out/rccl_bench.txt
bash tools/gpu_stream_ab.sh
