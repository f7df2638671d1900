"""Does an initialised RCCL process group slow the native step down? Same process, same device:
time the bare native ResNet-50 step, then init torch.distributed (nccl, eager, world 1) and our
RCCL communicator, and time the bare step again, then the DDP-wrapped step.
Usage (GPU box): python tools/pg_effect.py [--steps 20]"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(tr, steps, start):
    for i in range(3):
        tr.step(start + i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        tr.step(start + 3 + i)
    torch.cuda.synchronize()
    return round(1e3 * (time.perf_counter() - t0) / steps, 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from pytorch_distributed_amd.models.native import NativeTrainer
    tr = NativeTrainer("resnet50", 400, torch.bfloat16, dev)
    res = {"bare_no_pg": timed(tr, a.steps, 0)}
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29677", world_size=1, rank=0,
                            device_id=dev)
    res["bare_with_pg"] = timed(tr, a.steps, 100)
    from pytorch_distributed_amd.parallel.rccl import RcclCommunicator
    comm = RcclCommunicator(dev)
    res["bare_with_pg_and_comm"] = timed(tr, a.steps, 200)
    print(json.dumps(res), flush=True)
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
