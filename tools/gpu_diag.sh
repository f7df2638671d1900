#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python tools/diag_native.py resnet50 64 8 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python tools/diag_native.py resnet50 224 16 2>&1 | grep -v amdgpu.ids
