#!/bin/bash
set -o pipefail
export PDA_NO_BUILD=1   # the in-tree libraries travel with the snapshot (built on the CPU side)
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_native.py resnet50 64 8 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python tools/diag_native.py resnet50 224 16 2>&1 | grep -v amdgpu.ids
