#!/bin/bash
# GPU-box script: the GPU tests named in $TESTS (default: all), then bench.py (1 GPU) -> gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
if [ "${TESTS:-all}" != "none" ]; then
  T=${TESTS:-tests}; [ "$T" = all ] && T=tests
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
  rc=$?; tail -8 gpurun_out/pytest_quick.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -30 gpurun_out/bench_quick.err; exit 1; }
cat gpurun_out/bench_quick.json
