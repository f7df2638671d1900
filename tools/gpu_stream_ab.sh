#!/bin/bash
# GPU-box script: the step with the weight-gradient stream (default) vs everything on one stream
# (PDA_WGRAD_STREAM=0), alternating bench runs, then one kernel trace of each with the per-stream
# timeline (tools/stream_timeline.py) -> gpurun_out/stream_ab/.
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/stream_ab
mkdir -p $O
for rep in 1 2; do
  for v in 1 0; do
    PDA_WGRAD_STREAM=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 \
      --amp-steps 0 --dp-steps 0 > $O/bench_s$v.$rep.json 2> $O/bench_s$v.$rep.err || { tail -20 $O/bench_s$v.$rep.err; exit 1; }
    echo "stream=$v rep=$rep $(cat $O/bench_s$v.$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  PDA_WGRAD_STREAM=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_s$v -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --fp32-steps 0 --amp-steps 0 --dp-steps 0 > $O/prof_s$v.json 2> $O/prof_s$v.err || { tail -20 $O/prof_s$v.err; exit 1; }
  (cd $R && python tools/stream_timeline.py $O/prof_s$v > $O/timeline_s$v.txt && python tools/prof_summary.py $O/prof_s$v 7 > $O/summary_s$v.md; cat $O/timeline_s$v.txt)
done
