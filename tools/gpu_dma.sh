#!/bin/bash
# LDS-DMA conv tiles: numerics on the GPU, then the per-shape conv bench (all tiles).
set -o pipefail
mkdir -p gpurun_out
export PDA_NO_BUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_shapes_gpu.py -k "dma" > gpurun_out/dma_test.log 2>&1 || { tail -40 gpurun_out/dma_test.log; exit 1; }
tail -3 gpurun_out/dma_test.log
timeout -k 10 600 python -u tools/conv_bench.py 400 5 > gpurun_out/conv_bench_dma.txt 2>&1 || { tail -20 gpurun_out/conv_bench_dma.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/conv_bench_dma.txt
