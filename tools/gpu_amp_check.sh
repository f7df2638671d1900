#!/bin/bash
# GPU-box script: AMP tests + the bench's AMP pass (fp16 + dynamic loss scaling)
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/amp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_model_gpu.py -k "amp" -x -q --timeout 300 --timeout-method thread > gpurun_out/amp/tests.log 2>&1 || { tail -30 gpurun_out/amp/tests.log; exit 1; }
tail -2 gpurun_out/amp/tests.log
for r in 1 2; do
  timeout -k 10 600 python bench.py --fp32-steps 0 --dp-steps 0 > gpurun_out/amp/bench$r.json 2> gpurun_out/amp/bench$r.err || { tail -20 gpurun_out/amp/bench$r.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/amp/bench$r.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('amp_fp16_ms_per_step'), d.get('amp_loss_scale'))"
done
