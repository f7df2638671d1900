#!/bin/bash
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/entry
run() { tag=$1; shift; env "$@" timeout -k 10 300 python tools/ddp_sync_diag.py --steps 15 > gpurun_out/entry/$tag.txt 2>&1; rc=$?; echo "== $tag"; grep -E "^ddp_nosync|^bare_nosync" gpurun_out/entry/$tag.txt; [ $rc -ne 0 ] && { tail -20 gpurun_out/entry/$tag.txt; exit 1; }; return 0; }
run prio0 PDA_COMM_PRIO=0 || exit 1
run default || exit 1
run hwq3 GPU_MAX_HW_QUEUES=3 || exit 1
run hwq5 GPU_MAX_HW_QUEUES=5 || exit 1
run hwq6 GPU_MAX_HW_QUEUES=6 || exit 1
