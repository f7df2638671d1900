#!/bin/bash
# GPU-box script: rocprofv3 kernel traces (kernel-trace only) of the bf16 bench step under two
# environment settings, then tools/trace_cmp.py side by side.
# usage: A="PDA_X=0" B="PDA_X=1" [TAG=name] bash tools/gpu_trace_ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/trace_ab/${TAG:-ab}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp PDA_NO_BUILD=1
for v in A B; do
  envs=(); [ "${!v}" != "-" ] && IFS=, read -ra envs <<< "${!v}"
  for e in "${envs[@]}"; do export "$e"; done
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o p -- \
    python3 $R/bench.py --engine native --steps 5 --warmup 3 --fp32-steps 0 --amp-steps 0 --dp-steps 0 --util-steps 0 \
    > $O/$v.json 2> $O/$v.err || { echo "trace $v failed"; tail -20 $O/$v.err; exit 1; }
  for e in "${envs[@]}"; do unset "${e%%=*}"; done
done
cd $R && python tools/trace_cmp.py $O/A $O/B > $O/cmp.md && head -70 $O/cmp.md
