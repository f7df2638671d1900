"""Standalone reproducer for the HIP multi-queue graph-launch crash seen with DataParallel replay
(profiles/ab_r4.md section 7: a segfault inside hipGraphLaunch, an out-of-range read of a per-graph
stream list in libamdhip64.so, called from CUDAGraph::replay).

It records graphs in the SHAPE of parallel/dp.py _ReplicaGraph, with plain torch ops instead of the
native ResNet kernels:
  * a capture stream; the body forks to a second stream (wait_stream) and joins back inside the
    capture, as the native backward's weight-gradient stream does;
  * the capture is cut into several segment graphs that share ONE memory pool (capture_end /
    capture_begin(pool=...) mid-body), and in ``--side`` mode each segment's second-stream work is
    recorded as a graph of its own on the second stream;
  * replay: segment graphs on the caller's stream, side graphs on the second stream behind them,
    many iterations, optionally from a worker thread per replica (``--threads``).

Run it with DEBUG_HIP_FORCE_GRAPH_QUEUES unset (HIP's default: a graph's parallel branches launch
on internal streams) and =1 (one queue). Prints one JSON line (progress on stderr); a crash is the
HIP runtime's (the script uses only public torch APIs).
Round-5 results (profiles/ab_r5.md section 7): unset and =1 run clean in every configuration
(up to --threads 4 --segments 8 --side, 500 replays); =0 is NOT the default but zero graph queues:
it dies with SIGFPE inside capture_end (graph instantiation) even with --segments 1 --branches 0.
Usage: env -u DEBUG_HIP_FORCE_GRAPH_QUEUES python tools/graph_queue_repro.py [--side]
       [--threads N] [--segments S] [--iters I] [--branches B]"""
import argparse
import json
import os
import sys
import threading
import time

import torch


def body(x, ws, side, nseg, branches, cut, fork=True):
    """One 'step': per segment a chain of matmuls on the current stream, each fork-joined with
    ``branches`` matmul chains on the second stream (``fork``; else that work is left to the side
    graphs), joined back before ``cut(s)`` ends segment s."""
    cur = torch.cuda.current_stream()
    h = x
    for s in range(nseg):
        for _ in range(3):
            h = torch.tanh(h @ ws[0])
            if fork:
                for b in range(branches):
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        ws[2 + b].add_(h.t() @ h, alpha=1e-6)   # 'weight gradient' on the 2nd stream
            h = h @ ws[1]
        if fork and branches > 0:
            cur.wait_stream(side)
        cut(s)
    return h


class Replica:
    def __init__(self, dev, n, nseg, branches, side_split):
        self.dev = dev
        with torch.cuda.device(dev):
            self.x = torch.randn(n, n, device=dev)
            self.ws = [torch.randn(n, n, device=dev) / n ** 0.5 for _ in range(2 + branches)]
            self.side = torch.cuda.Stream(dev)
            self.graphs, self.sides = [], []
            cap = torch.cuda.Stream(dev)
            cur = torch.cuda.current_stream(dev)
            body(self.x, self.ws, self.side, nseg, branches, lambda s: None)   # warm-up, eager
            torch.cuda.synchronize(dev)
            print("warm-up done", file=sys.stderr, flush=True)
            cap.wait_stream(cur)
            self.side.wait_stream(cur)
            pool = [None]

            def cut(s):
                print(f"segment {s}: capture_end", file=sys.stderr, flush=True)
                self.graphs[-1].capture_end()
                print(f"segment {s}: instantiated", file=sys.stderr, flush=True)
                if pool[0] is None:
                    pool[0] = self.graphs[0].pool()
                if side_split:
                    # the second stream's queued work of this segment as a graph of its own
                    gs = torch.cuda.CUDAGraph()
                    with torch.cuda.stream(self.side):
                        gs.capture_begin(pool=pool[0])
                        for b in range(branches):
                            self.ws[2 + b].mul_(0.999)
                        gs.capture_end()
                    self.sides.append(gs)
                else:
                    self.sides.append(None)
                if s + 1 < nseg:
                    g2 = torch.cuda.CUDAGraph()
                    g2.capture_begin(pool=pool[0])
                    self.graphs.append(g2)
            with torch.cuda.stream(cap):
                g = torch.cuda.CUDAGraph()
                self.graphs.append(g)
                g.capture_begin()
                body(self.x, self.ws, self.side, nseg, branches, cut, fork=not side_split)
            cur.wait_stream(cap)
            cur.wait_stream(self.side)
            torch.cuda.synchronize(dev)

    def replay(self):
        with torch.cuda.device(self.dev):
            st = torch.cuda.current_stream(self.dev)
            for g, gs in zip(self.graphs, self.sides):
                g.replay()
                if gs is not None:
                    self.side.wait_stream(st)
                    with torch.cuda.stream(self.side):
                        gs.replay()
            st.wait_stream(self.side)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", action="store_true", help="record second-stream work as graphs of their own")
    ap.add_argument("--threads", type=int, default=0, help="replicas replayed from one thread each")
    ap.add_argument("--segments", type=int, default=4)
    ap.add_argument("--branches", type=int, default=2)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--n", type=int, default=256)
    a = ap.parse_args()
    t0 = time.time()
    dev = torch.device("cuda", 0)
    reps = [Replica(dev, a.n, a.segments, a.branches, a.side) for _ in range(max(1, a.threads))]
    print(f"captured {len(reps)} replica(s)", file=sys.stderr, flush=True)
    for it in range(a.iters):
        if it < 3:
            print(f"replay {it}", file=sys.stderr, flush=True)
        if a.threads > 1:
            ts = [threading.Thread(target=r.replay) for r in reps]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        else:
            for r in reps:
                r.replay()
        if it % 50 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    print(json.dumps({"ok": True, "queues_env": os.environ.get("DEBUG_HIP_FORCE_GRAPH_QUEUES"),
                      "side": a.side, "threads": a.threads, "segments": a.segments,
                      "branches": a.branches, "iters": a.iters,
                      "graphs_per_replica": len(reps[0].graphs) + sum(g is not None for g in reps[0].sides),
                      "s": round(time.time() - t0, 2)}))


if __name__ == "__main__":
    main()
