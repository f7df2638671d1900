"""Headline benchmark: ResNet-50 training images/sec, batch 400 per GPU, whole job.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is
launched by ``torch.distributed.run`` (one rank per GPU, RCCL over xGMI). Each
step is a full training step on synthetic data (on-device generation of the
batch, forward, loss, backward with bucketed gradient all-reduce, fused SGD with
momentum + weight decay), random-init ResNet-50, bf16 compute / fp32 master
weights. W untimed warm-up steps, then EXACTLY K timed steps bracketed by a
barrier + device synchronize on both sides; the MAX elapsed over ranks is used.
Rank 0 prints ONE JSON line.

Reference metric: images/sec whole node at bs 400/GPU; published
(derived) 717.0 img/s on 1 GPU and 5,546.7 img/s on 8 GPUs (AMP-DDP "Apex").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

BASELINE = {1: 717.0, 8: 5546.7}      # BASELINE.md derived images/sec (other hardware)
BASELINE_DP = {1: 717.0, 8: 1301.2}   # the nn.DataParallel bar of result.png
GRAPH_DEFAULT = os.environ.get("PDA_GRAPH", "0") == "1"


def _metric_name() -> str:
    """The headline metric exactly as BASELINE.json names it."""
    try:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except (OSError, ValueError, KeyError):
        return "images/sec (whole node) ResNet-50 bs=400 at 1/2/4/8 MI355X; scaling efficiency"


METRIC = _metric_name()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=400, help="per-GPU batch")
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--engine", default="auto", choices=["auto", "native", "torch"])
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--dp", action="store_true",
                    help="single-process DataParallel over --gpus devices (resnet_dp.py config)")
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the step in a HIP graph (1/0; default: on for 1 GPU, native engine)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    os.environ.setdefault("MX_WATCHDOG", "0")   # timed runs: no polling thread beside the step
    ndev = max(torch.cuda.device_count(), 1)
    device = torch.device("cuda", local_rank % ndev)   # >1 rank per GPU only in CPU-side rehearsals
    torch.cuda.set_device(device)
    if world > 1 and os.environ.get("PDA_BIND_NUMA", "1") != "0":
        # one rank per GPU, pinned to that GPU's NUMA node as the reference's
        # hfai.multiprocessing.spawn(bind_numa=True)
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from pytorch_distributed_amd.launch import bind_numa
        bind_numa(local_rank % ndev)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("PDA_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pytorch_distributed_amd.bench_step import make_trainer
    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.dtype]
    graph = args.graph == 1 or (args.graph < 0 and world == 1 and GRAPH_DEFAULT)
    if args.dp:
        if world > 1:
            raise SystemExit("--dp is one process driving --gpus devices; do not launch it with torchrun")
        from pytorch_distributed_amd.bench_step import make_dp_trainer
        tr = make_dp_trainer(args.arch, args.batch, dtype, args.gpus, args.image_size)
        world = args.gpus            # images/sec over all devices of the process
        sync_all = lambda: [torch.cuda.synchronize(d) for d in range(args.gpus)]  # noqa: E731
    else:
        tr = make_trainer(args.arch, args.batch, dtype, device, engine=args.engine,
                          world=world, rank=rank, bucket_mb=args.bucket_mb, image_size=args.image_size,
                          graph=graph)
        sync_all = torch.cuda.synchronize

    for i in range(args.warmup):
        tr.step(i)
    sync_all()
    multi_proc = world > 1 and not args.dp

    def barrier():
        if multi_proc:
            import torch.distributed as dist
            dist.barrier()
        sync_all()

    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        tr.step(args.warmup + i)
    barrier()
    elapsed = time.perf_counter() - t0
    if multi_proc:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss = tr.last_loss()
    ms = 1000.0 * elapsed / max(args.steps, 1)
    value = args.batch * world * args.steps / elapsed
    base = (BASELINE_DP if args.dp else BASELINE).get(world)
    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / base, 3) if base else None,
            "dtype": args.dtype,
            "data": "synthetic (on-device generated 3x224x224, random-init weights)",
            "config": {"model": args.arch, "global_batch": args.batch * world,
                       "per_gpu_batch": args.batch, "seq_len": None,
                       "parallelism": (f"dataparallel{world}" if args.dp else f"dp{world}"),
                       "engine": tr.engine,
                       "hip_graph": bool(getattr(tr, "graphed", None)),
                       "optimizer": "SGD(lr=0.1, momentum=0.9, wd=1e-4)"},
            "loss": loss,
            "max_mem_gb": round(torch.cuda.max_memory_allocated(device) / 1e9, 2),
        }
        print(json.dumps(rec), flush=True)
    if multi_proc:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
