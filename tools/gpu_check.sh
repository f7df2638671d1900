#!/bin/bash
# GPU-box script: GPU tests, smoke, default native bench (+ optional 2-rank rehearsal) -> gpurun_out/check/.
set -o pipefail
export PDA_NO_BUILD=1   # the in-tree libraries travel with the snapshot (built on the CPU side)
O=gpurun_out/check
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
rc=$?
tail -15 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 700 python bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
if [ -n "$REHEARSE2" ]; then
  PDA_DIST_BACKEND=gloo PDA_COMM=torch timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --rehearse-fold --steps 3 --warmup 1 --batch 64 \
    > $O/bench_rehearse2.json 2> $O/bench_rehearse2.err || { tail -30 $O/bench_rehearse2.err; exit 1; }
  cat $O/bench_rehearse2.json
fi
