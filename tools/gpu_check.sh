#!/bin/bash
# GPU-box script: build in-tree, run GPU tests, smoke, short native bench (+ optional 2-rank rehearsal).
set -o pipefail
export PDA_NO_BUILD=1   # the in-tree libraries travel with the snapshot (built on the CPU side)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -m pytest tests -m gpu -x -q --timeout 700 ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --engine native --steps 10 --warmup 3 > gpurun_out/bench_native.json 2> gpurun_out/bench_native.err || { tail -30 gpurun_out/bench_native.err; exit 1; }
cat gpurun_out/bench_native.json
if [ -n "$REHEARSE2" ]; then
  PDA_DIST_BACKEND=gloo PDA_COMM=torch timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 64 \
    > gpurun_out/bench_rehearse2.json 2> gpurun_out/bench_rehearse2.err || { tail -30 gpurun_out/bench_rehearse2.err; exit 1; }
  cat gpurun_out/bench_rehearse2.json
fi
