#!/bin/bash
# GPU-box script: rocprofv3 kernel traces of the round-1 tree (_r1/, a git worktree of 13df5b0
# with its own in-tree build) and of the current tree under env variants (PROF_VARIANTS: a list of
# VAR=value, default the current defaults), back to back on one device, for per-kernel regression
# hunting (tools/prof_cmp.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
run() {  # name dir envs...
  local name=$1 dir=$2; shift 2
  mkdir -p $R/gpurun_out/$name
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$name -o run -- \
    python3 $dir/bench.py --engine native --steps 6 --warmup 2 $EXTRA > $R/gpurun_out/$name/bench.json 2> $R/gpurun_out/$name/bench.err
}
run prof_r1 $R/_r1 PDA_X=1 || exit 1
EXTRA="--fp32-steps 0"
i=0
for v in ${PROF_VARIANTS:-PDA_X=1}; do
  i=$((i+1))
  run prof_$i $R $v || exit 1
done
