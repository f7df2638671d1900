#!/bin/bash
# GPU-box script: hardware counters of chosen conv launches, one counter group per run
# (kernel-trace only, never combined with sys/runtime tracing).
# usage: CASES="C16:fwd:1256:128 C16:fwd:-128:128" [PDA_KERNEL_LIB=...] bash tools/gpu_pmc_case.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_case
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp PDA_NO_BUILD=1
for c in $CASES; do
  IFS=: read shape ps bm bn <<< "$c"
  gi=0
  for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
    gi=$((gi+1))
    d=$OUT/${shape}_${ps}_${bm}_${bn}_g$gi
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $d -o p -- \
      python3 $R/tools/conv_one.py $shape $ps 3 $bm $bn >> $OUT/log.txt 2>&1 || { echo "pmc failed: $c / $grp"; tail -5 $OUT/log.txt; exit 1; }
  done
done
cd $R && python tools/pmc_summary.py $OUT | tee $OUT/summary.txt
