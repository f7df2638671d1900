#!/bin/bash
# GPU-box script: bench.py over a matrix of configs (dtype / engine / arch), one process each.
# usage: CONFIGS="--dtype bf16|--dtype fp16|--dtype fp32 --engine torch" bash tools/gpu_matrix.sh
set -o pipefail
mkdir -p gpurun_out/matrix
export PYTHONUNBUFFERED=1
IFS='|' read -ra CFG <<< "${CONFIGS:---dtype bf16}"
i=0
for c in "${CFG[@]}"; do
  i=$((i+1)); f=gpurun_out/matrix/m_$i
  timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} $c > $f.json 2> $f.err || { echo "FAIL [$c]"; tail -20 $f.err; exit 1; }
  echo "[$c] $(python -c "import json; r=json.load(open('$f.json')); print(r['value'], 'img/s', r['ms_per_step'], 'ms', r['config']['engine'], r['dtype'], r['config']['model'], 'loss', r['loss'], 'mem', r['max_mem_gb'])")"
done
