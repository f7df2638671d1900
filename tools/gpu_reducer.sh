set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_ddp_gpu.py tests/test_scripts_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_red.log 2>&1 || { tail -40 gpurun_out/pytest_red.log; exit 1; }
tail -12 gpurun_out/pytest_red.log
PDA_CPP_REDUCER=1 timeout -k 10 300 python tools/ddp_overhead.py --steps 20 > gpurun_out/ddp_ovh_cpp.txt 2>&1 || { tail -20 gpurun_out/ddp_ovh_cpp.txt; exit 1; }
PDA_CPP_REDUCER=0 timeout -k 10 300 python tools/ddp_overhead.py --steps 20 > gpurun_out/ddp_ovh_py.txt 2>&1 || { tail -20 gpurun_out/ddp_ovh_py.txt; exit 1; }
echo CPP; tail -3 gpurun_out/ddp_ovh_cpp.txt; echo PY; tail -3 gpurun_out/ddp_ovh_py.txt
