#!/bin/bash
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py tests/test_scripts_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ddpfix_tests.log 2>&1; rc=$?; tail -5 gpurun_out/ddpfix_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ddp_sync_diag.py --steps 15 > gpurun_out/ddpfix_diag.txt 2>&1 || { tail -20 gpurun_out/ddpfix_diag.txt; exit 1; }
grep -E "^(bare|ddp)" gpurun_out/ddpfix_diag.txt
bash tools/gpu_entry_steps.sh
