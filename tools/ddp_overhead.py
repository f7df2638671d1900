"""Per-step cost of the DDP wrapper at world size 1 (RCCL communicator, bucket all-reduces, buffer
sync) vs the bare native step -- what each rank pays on top of compute in the multi-GPU bench.
Usage (GPU box): python tools/ddp_overhead.py [--steps 20] [--comm native|torch]"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(tr, steps):
    for i in range(3):
        tr.step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        tr.step(3 + i)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--comm", default="native")
    a = ap.parse_args()
    os.environ["PDA_COMM"] = a.comm
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29655", world_size=1, rank=0,
                            device_id=dev)
    from pytorch_distributed_amd.models.native import NativeTrainer
    from pytorch_distributed_amd.parallel.ddp import DistributedDataParallel
    tr = NativeTrainer("resnet50", 400, torch.bfloat16, dev)
    bare = timed(tr, a.steps)
    tr.net = DistributedDataParallel(tr.model, bucket_cap_mb=32.0)
    wrapped = timed(tr, a.steps)
    print(json.dumps({"bare_ms": round(bare, 3), "ddp_ms": round(wrapped, 3), "comm": a.comm,
                      "communicator": type(tr.net.comm).__name__}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
