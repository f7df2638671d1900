#!/bin/bash
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/rccl
for v in "--op sum" "--op avg" "--op avg --backend nccl" "--op avg --backend nccl --device-id"; do
  tag=$(echo $v | tr -d ' -')
  timeout -k 10 120 python tools/rccl_bench.py --max-mb 64 --reps 5 $v > gpurun_out/rccl/$tag.txt 2>&1 || { tail -20 gpurun_out/rccl/$tag.txt; exit 1; }
  echo "== $v"; grep '"allreduce' gpurun_out/rccl/$tag.txt | tail -3
done
