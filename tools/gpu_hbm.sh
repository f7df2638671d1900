#!/bin/bash
# GPU-box script: HBM traffic of the native bench step -- FETCH_SIZE and WRITE_SIZE (derived TCC
# metrics, one pass each: together they exceed the 4 TCC counters of one pass), kernel-trace only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/hbm
cd /tmp && export TMPDIR=/tmp
for m in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $m --output-format csv -d $R/gpurun_out/hbm/$m -o p -- \
    python3 $R/bench.py --engine native --steps ${STEPS:-3} --warmup 2 --fp32-steps 0 --amp-steps 0 --dp-steps 0 --util-steps 0 \
    > $R/gpurun_out/hbm/$m.json 2> $R/gpurun_out/hbm/$m.err || { tail -20 $R/gpurun_out/hbm/$m.err; exit 1; }
done
cd $R && python tools/hbm_summary.py gpurun_out/hbm ${STEPS_TOTAL:-5} | tee gpurun_out/hbm/summary.md
