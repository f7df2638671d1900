"""Host-side enqueue time of one native training step (eager schedule vs HIP-graph replay).
The GPU is drained before each step, so the measured time is pure host work: what a
single-process multi-GPU driver (DataParallel) pays per device per step.
Usage (GPU box): python tools/host_overhead.py [--batch 400] [--arch resnet50]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--dp", type=int, default=0,
                    help="N>0: DataParallel with N graph-replayed replicas on cuda:0, serial vs "
                         "threaded replay enqueue (PDA_DP_THREADS)")
    a = ap.parse_args()
    if a.dp:
        return dp_overhead(a)
    from pytorch_distributed_amd.models.native import NativeTrainer
    dev = torch.device("cuda", 0)
    out = {}
    for graph in (False, True):
        tr = NativeTrainer(a.arch, a.batch, torch.bfloat16, dev, graph=graph)
        for i in range(3):
            tr.step(i)
        torch.cuda.synchronize()
        host, full = [], []
        for i in range(a.steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.step(3 + i)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            host.append(1e3 * (t1 - t0))
            full.append(1e3 * (t2 - t0))
        out["graph" if graph else "eager"] = {"host_enqueue_ms": round(min(host), 3),
                                              "step_ms": round(min(full), 3)}
        del tr
        torch.cuda.empty_cache()
    print(json.dumps({"arch": a.arch, "batch": a.batch, **out}))


def dp_overhead(a):
    from pytorch_distributed_amd.data import SyntheticImageNet
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    from pytorch_distributed_amd.parallel import DataParallel
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    dp = DataParallel(NativeResNet(build_model(a.arch), device=dev, image_size=224),
                      device_ids=[0] * a.dp)
    opt = dp.make_optimizer(lr=0.1, momentum=0.9, weight_decay=1e-4)
    gen = dp.module.input_generator(SyntheticImageNet("train", image_size=224))
    x, y = gen(torch.arange(a.batch * a.dp))
    out = {}
    for mode in ("1", "0"):   # threaded, serial
        os.environ["PDA_DP_THREADS"] = mode
        for i in range(2):
            dp.train_step(x, y, opt)
        torch.cuda.synchronize()
        host, full = [], []
        for i in range(a.steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dp.train_step(x, y, opt)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            host.append(1e3 * (t1 - t0))
            full.append(1e3 * (t2 - t0))
        out["threaded" if mode == "1" else "serial"] = {
            "host_enqueue_ms": round(min(host), 3), "step_ms": round(min(full), 3)}
    print(json.dumps({"arch": a.arch, "batch_per_replica": a.batch, "replicas": a.dp, **out}))


if __name__ == "__main__":
    main()
