#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python tools/conv_bench.py 400 5 > gpurun_out/conv_bench.txt 2>&1; rc=$?
cat gpurun_out/conv_bench.txt | grep -v amdgpu.ids
exit $rc
