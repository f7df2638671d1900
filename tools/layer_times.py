"""Where a native ResNet-50 step spends its time, by stage: HIP events at the engine's probe points
(after the stem and after every residual block, forward and backward) in steps run on ONE stream
(PDA_WGRAD_STREAM=0 by default, so an interval holds exactly the kernels of that part of the
network), averaged over the timed steps. Also prints the bytes of the stage's activations.

Usage (GPU box): python tools/layer_times.py [--steps 10] [--two-streams]"""
import argparse
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--two-streams", action="store_true")
    a = ap.parse_args()
    if not a.two_streams:
        os.environ["PDA_WGRAD_STREAM"] = "0"
    import torch
    from pytorch_distributed_amd.models.native import NativeTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = NativeTrainer("resnet50", a.batch, torch.bfloat16, dev)
    m = tr.model
    marks = []

    def probe(phase, name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        marks.append((phase, name, e))

    for i in range(3):
        tr.step(i)
    torch.cuda.synchronize()
    m.probe = probe
    acc = defaultdict(float)
    for i in range(a.steps):
        marks.clear()
        st = torch.cuda.Event(enable_timing=True)
        en = torch.cuda.Event(enable_timing=True)
        st.record()
        tr.step(3 + i)
        en.record()
        torch.cuda.synchronize()
        prev = ("start", "", st)
        for phase, name, e in marks:
            acc[(phase, name.split(".")[0])] += prev[2].elapsed_time(e)
            prev = (phase, name, e)
        acc[("rest", "head+loss / stem bwd+SGD")] += prev[2].elapsed_time(en) if marks else 0.0
        acc[("total", "")] += st.elapsed_time(en)
    m.probe = None
    out = {f"{p}:{n}": round(v / a.steps, 3) for (p, n), v in acc.items()}
    print(json.dumps({"streams": 2 if a.two_streams else 1, "ms": out}), flush=True)
    for k, v in out.items():
        print(f"{k:40s} {v:8.3f} ms")


if __name__ == "__main__":
    main()
