#!/bin/bash
# GPU-box script: alternating bench.py A/B over environment settings. VARIANTS = space-separated
# "NAME=VALUE[,NAME=VALUE...]" entries ("-" = no change); REPS rounds; 20 timed steps each;
# BENCH_ARGS are appended to every bench.py command (e.g. "--dp --gpus 1"), TAG prefixes the files.
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/ab
for rep in $(seq ${REPS:-2}); do
  for v in ${VARIANTS:--}; do
    envs=(); [ "$v" != "-" ] && IFS=, read -ra envs <<< "$v"
    tag=${TAG:-}$(echo "$v" | tr -c 'A-Za-z0-9.\n' '_')
    env "${envs[@]}" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --amp-steps 0 --dp-steps 0 ${BENCH_ARGS} > gpurun_out/ab/$tag.$rep.json 2> gpurun_out/ab/$tag.$rep.err || { tail -20 gpurun_out/ab/$tag.$rep.err; exit 1; }
    echo "$v rep=$rep $(python -c "import json; d=json.load(open('gpurun_out/ab/$tag.$rep.json')); print(d['value'], d['ms_per_step'])")"
  done
done
