#!/bin/bash
# GPU-box script: one variant kernel library (LIB=ab/libpda_kernels_NAME.so) -- its kernel tests,
# an alternating step A/B against the in-tree library, and the LDS-conflict counter group of every
# step kernel under the variant (output gpurun_out/ldsv/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p $R/gpurun_out/ldsv
PDA_KERNEL_LIB=$LIB timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_shape_gpu.py tests/test_determinism_gpu.py -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/ldsv/pytest.log 2>&1 || { tail -30 $R/gpurun_out/ldsv/pytest.log; exit 1; }
tail -3 $R/gpurun_out/ldsv/pytest.log
REPS=${REPS:-3} TAG=ldsv_ VARIANTS="- PDA_KERNEL_LIB=$LIB" bash tools/gpu_ab_env.sh || exit 1
cd /tmp && export TMPDIR=/tmp
export PDA_KERNEL_LIB=$LIB
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/ldsv/g2 -o p -- \
  python3 $R/bench.py --engine native --steps 2 --warmup 1 --fp32-steps 0 --amp-steps 0 --dp-steps 0 --util-steps 0 --diag-steps 0 --comm-probe 0 > $R/gpurun_out/ldsv/g2.json 2> $R/gpurun_out/ldsv/g2.err || { tail -20 $R/gpurun_out/ldsv/g2.err; exit 1; }
echo "pmc ok"
