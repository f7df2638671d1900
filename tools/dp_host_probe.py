"""Host enqueue time vs device time of the 1-device DataParallel step (ResNet-50, batch 400):
eager and replayed from the replica graphs (PDA_DP_FORCE_REPLAY path). A replay whose host time
per step approaches its device time cannot run ahead of the GPU, and every step then starts
with the device waiting for the first segment's graph launch.

    python tools/dp_host_probe.py [steps]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    from pytorch_distributed_amd.runtime.graphs import request_single_queue_graphs
    request_single_queue_graphs()   # (before HIP starts: the replica graphs need it)
    from pytorch_distributed_amd.bench_step import _DPTrainer
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    tr = _DPTrainer("resnet50", 400, torch.bfloat16, [0], 224)
    for mode in ("eager", "replay"):
        tr.dp.force_replay = mode == "replay"
        for i in range(4):
            tr.step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        host = []
        for i in range(steps):
            h0 = time.perf_counter()
            tr.step(100 + i)
            host.append(time.perf_counter() - h0)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.sort()
        print(f"{mode:7s} host enqueue {1e3 * (t1 - t0) / steps:7.2f} ms/step (median step "
              f"{1e3 * host[len(host) // 2]:6.2f}, max {1e3 * host[-1]:6.2f}); wall incl. drain "
              f"{1e3 * (t2 - t0) / steps:7.2f} ms/step")
        if mode == "replay":
            rg = tr.dp._graphs[0]
            print(f"        segments {len(rg.graphs)}, side graphs {sum(g is not None for g in rg.sides)}")
    print("dp_host_probe: ok")


if __name__ == "__main__":
    main()
