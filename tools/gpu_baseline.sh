#!/bin/bash
# GPU-box script: PyTorch-ROCm (MIOpen) reference bench for comparison.
set -o pipefail
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 600 python bench.py --engine torch --steps 10 --warmup 5 > gpurun_out/bench_torch.json 2> gpurun_out/bench_torch.err
