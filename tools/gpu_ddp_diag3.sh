#!/bin/bash
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/entry
run() { tag=$1; shift; env "$@" timeout -k 10 300 python tools/ddp_sync_diag.py --steps 15 > gpurun_out/entry/$tag.txt 2>&1; rc=$?; echo "== $tag"; grep -E "^ddp_nosync|^bare_nosync" gpurun_out/entry/$tag.txt; [ $rc -ne 0 ] && { tail -20 gpurun_out/entry/$tag.txt; exit 1; }; return 0; }
run hwq8 GPU_MAX_HW_QUEUES=8 || exit 1
run nowgrad PDA_WGRAD_STREAM=0 || exit 1
run hwq2 GPU_MAX_HW_QUEUES=2 || exit 1
