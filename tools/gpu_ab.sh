#!/bin/bash
# GPU-box script: targeted GPU tests + A/B bench of env toggles (one process per variant).
# usage: TESTS="tests/x.py" VARIANTS="A=0,B=1 A=1,B=1" bash tools/gpu_ab.sh  (comma = several vars)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -m pytest $TESTS -m gpu -x -q --timeout 300 > gpurun_out/pytest_ab.log 2>&1
  rc=$?; tail -15 gpurun_out/pytest_ab.log; [ $rc -ne 0 ] && exit $rc
fi
i=0
for v in ${VARIANTS:-BASE=1}; do
  i=$((i+1)); f=gpurun_out/ab_$i
  env ${v//,/ } timeout -k 10 300 python bench.py --engine native --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS} > $f.json 2> $f.err || { echo "FAIL $v"; tail -20 $f.err; exit 1; }
  echo "$v $(python -c "import json,sys; r=json.load(open('$f.json')); print(r['value'], r['ms_per_step'], r['loss'])")"
done
