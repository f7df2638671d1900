#!/bin/bash
# GPU-box script: rocprofv3 kernel trace of the whole-step graph replay (bench.py --graph 1) with the
# per-stream timeline -- compare with tools/gpu_trace2.sh (eager).
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/trace_graph
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --graph 1 --steps 5 --warmup 3 --fp32-steps 0 --amp-steps 0 --dp-steps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cd $R && python tools/stream_timeline.py $O/prof > $O/timeline.txt && python tools/prof_summary.py $O/prof 7 > $O/summary.md && cat $O/timeline.txt && head -30 $O/summary.md && grep -o '"ms_per_step": [0-9.]*' $O/bench.json
