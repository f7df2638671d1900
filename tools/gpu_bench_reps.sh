#!/bin/bash
# GPU-box script: REPS full default bench.py runs back to back (every pass), one JSON each ->
# gpurun_out/benchreps/, with the headline / AMP / DataParallel / replay / fp32 keys printed.
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
O=gpurun_out/benchreps; mkdir -p $O
for i in $(seq ${REPS:-3}); do
  timeout -k 10 600 python -u bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -30 $O/bench_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$i.json')); print($i, {k: d.get(k) for k in ('value', 'ms_per_step', 'amp_fp16_images_per_sec', 'dp_images_per_sec', 'dp_replay_vs_eager', 'fp32_images_per_sec', 'fp32_exact_images_per_sec')})"
done
