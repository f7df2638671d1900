#!/bin/bash
set -o pipefail
export PDA_NO_BUILD=1   # the in-tree libraries travel with the snapshot (built on the CPU side)
mkdir -p gpurun_out
timeout -k 10 900 python tools/conv_bench.py 400 5 > gpurun_out/conv_bench.txt 2>&1; rc=$?
cat gpurun_out/conv_bench.txt | grep -v amdgpu.ids
exit $rc
