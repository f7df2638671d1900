#!/bin/bash
# GPU-box script (round 6): smoke, the named GPU tests, bench.py, then a rocprofv3 kernel trace of
# the bench step with the per-stream timeline -> gpurun_out/r6/.
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r6}
mkdir -p $O
if [ "${SMOKE:-1}" = 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
  tail -6 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  tail -25 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
if [ "${PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $R/bench.py --engine native --steps 5 --warmup 2 --fp32-steps 0 --amp-steps 0 --dp-steps 0 ${PROF_ARGS} > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
  cd $R
  python tools/prof_summary.py $O/prof 7 > $O/prof_summary.md && python tools/stream_timeline.py $O/prof > $O/timeline.txt && python tools/main_stream_summary.py $O/prof > $O/main_stream.txt
  head -45 $O/prof_summary.md; cat $O/timeline.txt; head -30 $O/main_stream.txt
fi
