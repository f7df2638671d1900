set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5p
timeout -k 10 300 python -u -m pytest tests/test_native_model_gpu.py -k "tail_fold_is_bit_exact or stem_wgrad_bna" -x -q --timeout 200 --timeout-method thread > gpurun_out/r5p/tests.log 2>&1; rc=$?
grep -E "AssertionError|assert |passed|failed" gpurun_out/r5p/tests.log | head -20
exit $rc
