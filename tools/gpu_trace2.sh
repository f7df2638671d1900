#!/bin/bash
# GPU-box script: one rocprofv3 kernel trace of the default (two-stream) bench step + summaries.
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/trace2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --fp32-steps 0 --amp-steps 0 --dp-steps 0 --util-steps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cd $R && python tools/stream_timeline.py $O/prof > $O/timeline.txt && python tools/prof_summary.py $O/prof 7 > $O/summary.md && cat $O/timeline.txt && head -30 $O/summary.md
