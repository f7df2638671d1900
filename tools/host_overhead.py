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
    a = ap.parse_args()
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


if __name__ == "__main__":
    main()
