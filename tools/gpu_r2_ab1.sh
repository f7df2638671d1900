#!/bin/bash
# round-2 A/B: in-launch BN reductions x MFMA shape (one process per variant) + kernel tests
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_conv_shapes_gpu.py tests/test_native_model_gpu.py tests/test_determinism_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_mf16.log 2>&1
tail -3 gpurun_out/pytest_mf16.log
PDA_MFMA=32 timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_conv_shapes_gpu.py tests/test_determinism_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_mf32.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_mf32.log
VARIANTS="PDA_INLAUNCH_BN=1,PDA_MFMA=16 PDA_INLAUNCH_BN=0,PDA_MFMA=16 PDA_INLAUNCH_BN=fwd,PDA_MFMA=16 PDA_INLAUNCH_BN=bwd,PDA_MFMA=16 PDA_INLAUNCH_BN=0,PDA_MFMA=32 PDA_INLAUNCH_BN=1,PDA_MFMA=32" BENCH_ARGS="--fp32-steps 0" bash tools/gpu_ab.sh
