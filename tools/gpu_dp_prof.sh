#!/bin/bash
# GPU-box script: kernel traces of the 1-device DataParallel step, replayed from the replica graphs
# (PDA_DP_FORCE_REPLAY=1) and eager (PDA_FORK_TRACK=0: the profiler's completion signalling makes
# tracked launches look slower), each with the stream timeline and the main-stream sequence.
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
R=$(pwd)
for v in replay eager; do
  O=gpurun_out/dpprof/$v; mkdir -p $R/$O
  # (eager: the plain one-device step, which is what DataParallel(1) runs; a --dp run would also
  # hold the forced-replay steps it times after its headline)
  if [ $v = replay ]; then export PDA_DP_FORCE_REPLAY=1; A="--dp"; else unset PDA_DP_FORCE_REPLAY; A="--dp-steps 0"; fi
  (cd /tmp && export TMPDIR=/tmp PDA_FORK_TRACK=0 && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py $A --gpus 1 --steps 5 --warmup 3 --fp32-steps 0 --amp-steps 0 > $R/$O/bench.json 2> $R/$O/bench.err) || { tail -20 $R/$O/bench.err; exit 1; }
  python tools/stream_timeline.py $O/prof > $O/timeline.txt && python tools/step_sequence.py $O/prof > $O/seq.txt && python tools/main_stream_summary.py $O/prof > $O/main.txt || exit 1
  echo "== $v"; cat $O/timeline.txt; tail -2 $O/seq.txt
done
