#!/bin/bash
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_native_model_gpu.py tests/test_determinism_gpu.py tests/test_graph_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dsapply_tests.log 2>&1; rc=$?; tail -3 gpurun_out/dsapply_tests.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/dsapply_tests.log; exit $rc; }
VARIANTS="- PDA_DS_APPLY_SIDE=0" REPS=4 bash tools/gpu_ab_env.sh
