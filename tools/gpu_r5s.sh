set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5s
timeout -k 10 900 python -u -m pytest tests/test_native_model_gpu.py tests/test_production_shape_gpu.py tests/test_determinism_gpu.py tests/test_dp_gpu.py tests/test_graph_gpu.py tests/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s/tests.log 2>&1 || { tail -30 gpurun_out/r5s/tests.log; exit 1; }
tail -2 gpurun_out/r5s/tests.log
VARIANTS="- PDA_FORK_TRACK=0" REPS=3 TAG=r5s_ bash tools/gpu_ab_env.sh || exit 1
A="PDA_FORK_TRACK=0" B="-" TAG=trk bash tools/gpu_trace_ab.sh > /dev/null 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python /root/repo/tools/trace_cmp.py gpurun_out/trace_ab/trk/A gpurun_out/trace_ab/trk/B | head -3
