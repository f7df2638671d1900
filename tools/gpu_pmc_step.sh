#!/bin/bash
# GPU-box script: hardware counters of every kernel of the bench step (the step's own shapes and
# operands; rocprofv3 serialises dispatches while collecting, so each kernel is measured alone),
# one counter group per run, kernel-trace only (never combined with sys/runtime tracing), plus the
# FETCH_SIZE / WRITE_SIZE calibration on a known byte count (tools/fetch_calib.py).
# Output: gpurun_out/pmc_step/summary.md (tools/pmc_step_summary.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_step
mkdir -p $O
cd /tmp && export TMPDIR=/tmp PDA_NO_BUILD=1
BENCH="$R/bench.py --engine native --steps 2 --warmup 1 --fp32-steps 0 --amp-steps 0 --dp-steps 0 --util-steps 0 --diag-steps 0 --comm-probe 0"
gi=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  gi=$((gi+1))
  echo "group $gi: $grp" | tee -a $O/log.txt
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/g$gi -o p -- \
    python3 $BENCH > $O/g$gi.json 2>> $O/log.txt || { echo "pmc failed: group $gi"; tail -20 $O/log.txt; exit 1; }
done
for m in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $m --output-format csv -d $O/calib_$m -o p -- \
    python3 $R/tools/fetch_calib.py > $O/calib_$m.txt 2>> $O/log.txt || { echo "calib failed: $m"; tail -20 $O/log.txt; exit 1; }
done
cd $R && python tools/pmc_step_summary.py $O > $O/summary.md && head -80 $O/summary.md
