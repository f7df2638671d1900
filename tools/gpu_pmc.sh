#!/bin/bash
# GPU-box script: hardware counters for representative conv kernels (counters in their own run,
# kernel-trace only -- never combined with sys/runtime tracing).
set -o pipefail
export PDA_NO_BUILD=1   # the in-tree libraries travel with the snapshot (built on the CPU side)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc/counters_list.txt 2>&1 || true
for case in "C16 fwd" "C3 fwd" "C16 dgrad" "C16 wgrad" "C4 dgrad"; do
  set -- $case
  gi=0
  for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    gi=$((gi+1))
    timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $R/gpurun_out/pmc/$1_$2_g$gi -o p -- \
      python3 $R/tools/conv_one.py $1 $2 3 >> $R/gpurun_out/pmc/log.txt 2>&1 || { echo "pmc failed for $case / $grp"; tail -5 $R/gpurun_out/pmc/log.txt; }
  done
done
cd $R && python tools/pmc_summary.py gpurun_out/pmc | tee gpurun_out/pmc/summary.txt
