set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp PDA_NO_BUILD=1
for c in C2 C10; do
  gi=0
  for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
             "FETCH_SIZE"; do
    gi=$((gi+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/${c}_g$gi -o p -- \
      python3 $R/tools/wgrad_tap_one.py $c tap 3 >> $O/log.txt 2>&1 || { echo "pmc failed: $c $gi"; tail -5 $O/log.txt; exit 1; }
  done
done
cd $R && PMC_KERNEL=wgrad_tap python tools/pmc_summary.py $O | tee $O/summary.txt
