#!/bin/bash
# GPU-box script: why the DDP entrypoint's step is slower than the single-GPU one at world 1.
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1 MASTER_IP=127.0.0.1 MX_NPROCS=1
mkdir -p gpurun_out/entry
python - <<'PY'
import os, sys
sys.path.insert(0, ".")
from pytorch_distributed_amd.launch import _gpu_numa_cpus
print("allowed cpus:", len(os.sched_getaffinity(0)), "gpu0 numa cpus:", (lambda c: (len(c), c[:4], c[-4:]) if c else None)(_gpu_numa_cpus(0)), "nproc", os.cpu_count())
PY
N=300
run() {
  tag=$1; s=$2; shift 2
  env "$@" MX_EPOCHS=1 MX_STEPS_PER_EPOCH=$N MX_VAL_STEPS=1 MX_SAVE_PATH=/tmp/entry_$tag \
    timeout -k 10 300 python $s > gpurun_out/entry/$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 gpurun_out/entry/$tag.log; exit 1; }
  t=$(grep "cost time" gpurun_out/entry/$tag.log | awk '{print $5}')
  echo "$tag: $(python -c "print(round(1000*$t/$N,2))") ms/step"
}
run ddp_default restnet_ddp.py MX_DTYPE=bf16 || exit 1
run ddp_nowatchdog restnet_ddp.py MX_DTYPE=bf16 MX_WATCHDOG=0 || exit 1
run ddp_nonuma restnet_ddp.py MX_DTYPE=bf16 PDA_BIND_NUMA=0 || exit 1
run ddp_nonuma_nowd restnet_ddp.py MX_DTYPE=bf16 PDA_BIND_NUMA=0 MX_WATCHDOG=0 || exit 1
run single restnet_ddp.py MX_DTYPE=bf16 PDA_BIND_NUMA=0 MX_WATCHDOG=0 PDA_COMM=torch || exit 1
timeout -k 10 200 python tools/ddp_overhead.py --steps 20 > gpurun_out/entry/ddp_overhead.txt 2>&1 && tail -1 gpurun_out/entry/ddp_overhead.txt
