set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5q
timeout -k 10 120 python tools/fork_bench.py 200 40 2>&1 | tee gpurun_out/r5q/fork.txt || exit 1
timeout -k 10 120 python tools/fork_bench.py 200 80 2>&1 | tee -a gpurun_out/r5q/fork.txt || exit 1
