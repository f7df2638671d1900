"""DDP (native RCCL communicator, world 1) step time with and without a per-step synchronize, and
the host time spent inside each phase of the step -- isolates host-side blocking in the DDP path.
Usage (GPU box): python tools/ddp_sync_diag.py [--steps 20] [--device-id]"""
import argparse
import json
import os
import sys
import time
from collections import defaultdict

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--device-id", action="store_true")
    ap.add_argument("--port", type=int, default=29656)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    kw = {"device_id": dev} if a.device_id else {}
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{a.port}", world_size=1, rank=0, **kw)
    from pytorch_distributed_amd.models.native import NativeTrainer
    from pytorch_distributed_amd.parallel.ddp import DistributedDataParallel
    tr = NativeTrainer("resnet50", 400, torch.bfloat16, dev)
    res = {}
    for wrap in (False, True):
        if wrap:
            tr.net = DistributedDataParallel(tr.model, bucket_cap_mb=32.0)
        for sync in (False, True):
            host = defaultdict(float)
            for i in range(3):
                tr.step(i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                ids = torch.arange(tr.batch, dtype=torch.int64) + (i + 3) * tr.batch
                h0 = time.perf_counter()
                x, y = tr.gen(ids)
                out = tr.net(x)
                loss = tr.crit(out, y)
                h1 = time.perf_counter()
                loss.backward()
                h2 = time.perf_counter()
                tr.opt.step()
                tr.opt.zero_grad()
                h3 = time.perf_counter()
                if sync:
                    torch.cuda.synchronize()
                h4 = time.perf_counter()
                host["fwd"] += h1 - h0
                host["bwd"] += h2 - h1
                host["opt"] += h3 - h2
                host["sync"] += h4 - h3
            torch.cuda.synchronize()
            ms = 1e3 * (time.perf_counter() - t0) / a.steps
            key = f"{'ddp' if wrap else 'bare'}_{'sync' if sync else 'nosync'}"
            res[key] = {"ms": round(ms, 2), **{k: round(1e3 * v / a.steps, 2) for k, v in host.items()}}
            print(key, json.dumps(res[key]), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
