#!/bin/bash
# GPU-box script (round 3, final tree): GPU suite, smoke, bench, per-stage times (1 and 2 streams).
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
bash tools/gpu_check.sh || exit $?
timeout -k 10 240 python tools/layer_times.py --steps 10 > gpurun_out/layer_times_s1.txt 2>&1 || { tail -20 gpurun_out/layer_times_s1.txt; exit 1; }
timeout -k 10 240 python tools/layer_times.py --steps 10 --two-streams > gpurun_out/layer_times_s2.txt 2>&1 || { tail -20 gpurun_out/layer_times_s2.txt; exit 1; }
grep -v "^{" gpurun_out/layer_times_s2.txt | tail -12
