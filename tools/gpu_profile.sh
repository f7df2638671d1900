#!/bin/bash
# GPU-box script: rocprofv3 kernel trace + stats of the native bench step.
set -o pipefail
export PDA_NO_BUILD=1   # the in-tree libraries travel with the snapshot (built on the CPU side)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- \
  python3 $R/bench.py --engine native --steps ${STEPS:-5} --warmup 2 --fp32-steps 0 --amp-steps 0 --dp-steps 0 ${BENCH_ARGS} > $R/gpurun_out/prof/bench.json 2> $R/gpurun_out/prof/bench.err || { tail -20 $R/gpurun_out/prof/bench.err; exit 1; }
cd $R && python tools/prof_summary.py gpurun_out/prof ${STEPS_TOTAL:-7} > gpurun_out/prof/summary.md && cat gpurun_out/prof/summary.md | head -60
