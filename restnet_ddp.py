"""ResNet-50, multi-process DDP (reference: restnet_ddp.py -- file name kept, typo included).

Launch once per node: MASTER_IP, MASTER_PORT, WORLD_SIZE (= #nodes), RANK (= node index);
one process per visible GPU is spawned (NUMA-bound). torchrun launches also work.
"""
import os
import sys

from pytorch_distributed_amd.config import config_for, parse_cli
from pytorch_distributed_amd.launch import spawn
from pytorch_distributed_amd.trainer import run


def main(local_rank, script="ddp", nprocs=None):
    run(config_for(script), mode=script, local_rank=local_rank, nprocs=nprocs)


def launch(script="ddp"):
    os.environ.update(parse_cli(sys.argv[1:]))   # optional flags -> MX_* env (inherited by ranks)
    if "LOCAL_RANK" in os.environ:            # started by torchrun
        lr = int(os.environ["LOCAL_RANK"])
        if os.environ.get("PDA_BIND_NUMA", "1") != "0":
            from pytorch_distributed_amd.launch import bind_numa
            bind_numa(lr)                     # before any HIP call (sysfs only)
        main(lr, script)
        return
    from pytorch_distributed_amd.launch import visible_gpu_count
    # counted from sysfs: no HIP call before each rank binds its NUMA node
    nprocs = int(os.environ.get("MX_NPROCS", "0")) or max(visible_gpu_count(), 1)
    spawn(main, args=(script, nprocs), nprocs=nprocs, bind_numa=True)


if __name__ == "__main__":
    launch("ddp")
