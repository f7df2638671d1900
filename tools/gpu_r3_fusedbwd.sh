#!/bin/bash
# GPU-box script: the one-launch BN-backward finalize + apply -- kernel test, model-level tests,
# then an alternating bench A/B against the two-launch path (PDA_FUSED_BWD=0).
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/fused
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "fused_matches_two_launches or bn_backward or dgrad_fused" -x -q --timeout 240 --timeout-method thread > gpurun_out/fused/kern.log 2>&1; rc=$?; tail -3 gpurun_out/fused/kern.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/fused/kern.log; exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_native_model_gpu.py tests/test_determinism_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fused/model.log 2>&1; rc=$?; tail -3 gpurun_out/fused/model.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/fused/model.log; exit $rc; }
for rep in 1 2; do
  for v in 1 0; do
    PDA_FUSED_BWD=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --amp-steps 0 --dp-steps 0 > gpurun_out/fused/b$v.$rep.json 2> gpurun_out/fused/b$v.$rep.err || { tail -20 gpurun_out/fused/b$v.$rep.err; exit 1; }
    echo "fused=$v rep=$rep $(python -c "import json; d=json.load(open('gpurun_out/fused/b$v.$rep.json')); print(d['value'], d['ms_per_step'])")"
  done
done
