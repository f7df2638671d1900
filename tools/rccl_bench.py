"""RCCL collective latency / bandwidth sweep on the native communicator (the alpha and the
per-byte cost of parallel/reducer.py's cost model). One process per GPU; on a 1-GPU box it runs at
world 1, where it measures the fixed cost of a collective (launch + RCCL kernel + event) and the
local copy bandwidth of the in-place all-reduce -- the link term needs the driver's 8-GPU run.

Each size: W untimed warmups, then R back-to-back collectives on the comm stream bracketed by HIP
events; reports the median of 5 such rounds. Also the in-process group (ncclCommInitAll) used by
DataParallel.

Usage: python tools/rccl_bench.py [--max-mb 128] [--reps 20]
       (world > 1: torch.distributed.run --nproc-per-node N tools/rccl_bench.py)"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, stream, reps):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(5):
        st.record(stream)
        for _ in range(reps):
            fn()
        en.record(stream)
        en.synchronize()
        out.append(st.elapsed_time(en) / reps)
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-mb", type=float, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--op", default="sum", choices=["sum", "avg"])
    ap.add_argument("--backend", default="gloo", help="torch.distributed backend of the rendezvous")
    ap.add_argument("--device-id", action="store_true",
                    help="pass device_id: torch creates ITS NCCL communicator eagerly (nccl backend)")
    a = ap.parse_args()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29681")
    kw = {"device_id": dev} if a.device_id else {}
    dist.init_process_group(a.backend, rank=rank, world_size=world, **kw)
    from pytorch_distributed_amd.parallel.rccl import RcclCommunicator, RcclGroup
    comm = RcclCommunicator(dev)
    sizes = []
    s = 4096
    while s <= a.max_mb * (1 << 20):
        sizes.append(s)
        s *= 4
    buf = torch.zeros(int(a.max_mb * (1 << 20)) // 4, dtype=torch.float32, device=dev)
    rows = []
    with torch.cuda.stream(comm.stream):
        for nbytes in sizes:
            t = buf[:nbytes // 4]
            for _ in range(3):
                comm.all_reduce(t, op=a.op)
            ms = timeit(lambda: comm.all_reduce(t, op=a.op), comm.stream, a.reps)
            # bus bandwidth convention: 2 (n-1)/n S / t; at world 1 the algorithm bandwidth S / t
            algbw = nbytes / (ms * 1e-3) / 1e9
            busbw = algbw * (2 * (world - 1) / world if world > 1 else 1.0)
            rows.append({"op": f"allreduce_{a.op}", "bytes": nbytes, "us": round(ms * 1e3, 2),
                         "algbw_GBs": round(algbw, 1), "busbw_GBs": round(busbw, 1)})
    if world == 1:
        grp = RcclGroup([local])
        for nbytes in sizes:
            t = buf[:nbytes // 4]
            for _ in range(3):
                grp.all_reduce([t])
            ms = timeit(lambda: grp.all_reduce([t]), torch.cuda.current_stream(dev), a.reps)
            rows.append({"op": "group_allreduce", "bytes": nbytes, "us": round(ms * 1e3, 2),
                         "algbw_GBs": round(nbytes / (ms * 1e-3) / 1e9, 1)})
        grp.close()
    # alpha / beta fit on the all-reduce rows: t = alpha + S / bw (least squares over the sizes)
    ar = [r for r in rows if r["op"].startswith("allreduce")]
    xs = [r["bytes"] for r in ar]
    ys = [r["us"] for r in ar]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    beta = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    alpha = my - beta * mx
    if rank == 0:
        for r in rows:
            print(json.dumps(r), flush=True)
        print(json.dumps({"fit": "t = alpha + S / bw", "world": world, "alpha_us": round(alpha, 2),
                          "bw_GBs": round(1e-3 / beta, 1) if beta > 0 else None,
                          "rccl_world": comm.rccl_count}), flush=True)
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
