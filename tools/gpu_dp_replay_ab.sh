#!/bin/bash
# GPU-box script: alternating `bench.py --dp --gpus 1` runs over environment variants, printing the
# eager step, the replica-graph replay step (dp_replay_ms_per_step) and their ratio per run.
# usage: REPS=2 VARIANTS="- PDA_WGRAD_SCALE=0.7" bash tools/gpu_dp_replay_ab.sh
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/dpab
for rep in $(seq ${REPS:-2}); do
  for v in ${VARIANTS:--}; do
    envs=(); [ "$v" != "-" ] && IFS=, read -ra envs <<< "$v"
    tag=$(echo "$v" | tr -c 'A-Za-z0-9.\n' '_')
    f=gpurun_out/dpab/$tag.$rep
    env "${envs[@]}" timeout -k 10 300 python bench.py --dp --gpus 1 --steps 20 --warmup 5 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
    echo "$v rep=$rep $(python -c "import json; d=json.load(open('$f.json')); print(d['ms_per_step'], d.get('dp_replay_ms_per_step'), d.get('dp_replay_vs_eager'))")"
  done
done
