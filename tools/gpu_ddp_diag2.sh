#!/bin/bash
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/entry
timeout -k 10 300 python tools/ddp_sync_diag.py --steps 15 > gpurun_out/entry/sync_diag.txt 2>&1; rc=$?; grep -E "^(bare|ddp)" gpurun_out/entry/sync_diag.txt; [ $rc -ne 0 ] && { tail -20 gpurun_out/entry/sync_diag.txt; exit 1; }
timeout -k 10 300 python tools/ddp_sync_diag.py --steps 15 --device-id > gpurun_out/entry/sync_diag_devid.txt 2>&1; rc=$?; grep -E "^(bare|ddp)" gpurun_out/entry/sync_diag_devid.txt; [ $rc -ne 0 ] && { tail -20 gpurun_out/entry/sync_diag_devid.txt; exit 1; }
exit 0
