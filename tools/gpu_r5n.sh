set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5n
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r5n/smoke.log 2>&1 || { tail -20 gpurun_out/r5n/smoke.log; exit 1; }
tail -1 gpurun_out/r5n/smoke.log
timeout -k 10 900 python bench.py > gpurun_out/r5n/bench.json 2> gpurun_out/r5n/bench.err || { tail -30 gpurun_out/r5n/bench.err; exit 1; }
cat gpurun_out/r5n/bench.json
