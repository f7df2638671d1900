"""Headline benchmark: ResNet-50 training images/sec, batch 400 per GPU, whole job.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it runs one rank
per GPU (RCCL over xGMI) -- launched by ``torch.distributed.run`` (``WORLD_SIZE`` must then equal
N), or, started bare, it launches the N ranks itself as a child ``torch.distributed.run`` after
checking that N GPUs are visible (fewer: a non-zero exit, never a silent smaller run). Each
step is a full training step on synthetic data (on-device generation of the
batch, forward, loss, backward with bucketed gradient all-reduce, fused SGD with
momentum + weight decay), random-init ResNet-50, bf16 compute / fp32 master
weights. W untimed warm-up steps, then EXACTLY K timed steps bracketed by a
barrier + device synchronize on both sides; the MAX elapsed over ranks is used.
Rank 0 prints ONE JSON line.

Self-validation for N > 1 (everything below runs AFTER the timed region):

* ``rccl_world``: the rank count RCCL itself reports for the gradient communicator
  (``ncclCommCount``), next to ``n_gpus`` from the launcher;
* ``buckets`` / ``bucket_bytes``: the gradient-bucket plan (identical on every rank:
  DistributedDataParallel verifies it across ranks at construction);
* ``exposed_comm_ms`` / ``bucket_allreduce_ms``: ``--diag-steps`` extra steps with HIP
  timing events around every bucket all-reduce and at the end of backward; exposed =
  backward end -> last bucket done (the part of communication NOT hidden by backward);
* ``weights_consistent``: a bit-exact checksum of the parameters and momentum buffers,
  all-reduced MIN and MAX over ranks; a mismatch (ranks that silently diverged) makes
  the run exit non-zero. ``PDA_BENCH_PERTURB_RANK=r`` perturbs rank r (test hook);
* finite rendezvous / RCCL-init timeouts (``PDA_DIST_TIMEOUT_S``), so a missing rank is
  an error, not a hang.

``fp32_images_per_sec``: a short pass of the same step in fp32 (the reference scripts'
precision) on the fp32 default -- f32 tensors with the convolutions on the bf16 MFMA as a hi/lo
three-term split (~16 significant bits per product; every conv pass at or below the error of the
TF32 convolutions the reference's fp32 runs use, tests/test_f32_precision_gpu.py) -- so the
like-for-like number is measured in the same run; and ``fp32_exact_images_per_sec``: the same f32
step on the exact f32 MFMA. For N > 1 each rank runs them without gradient all-reduce (per-GPU
fp32 compute, aggregated).

Reference metric: images/sec whole node at bs 400/GPU; published
(derived) 717.0 img/s on 1 GPU (fp32/TF32) and 5,546.7 img/s on 8 GPUs (AMP-DDP "Apex").
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import statistics
import sys
import time
import traceback

import torch

from pytorch_distributed_amd.utils.gpu_util import BusySampler, kernel_busy

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
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: rehearsal of the launch/validation contract without a GPU")
    ap.add_argument("--dp", action="store_true",
                    help="single-process DataParallel over --gpus devices (resnet_dp.py config)")
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the step in a HIP graph (1/0; default off, PDA_GRAPH=1 turns it "
                         "on for 1 GPU)")
    ap.add_argument("--diag-steps", type=int, default=3,
                    help="N>1: extra untimed steps with bucket timing events")
    ap.add_argument("--comm-probe", type=int, default=1,
                    help="N>1: measure all-reduce latency / bus bandwidth of the gradient "
                         "communicator after the timed region (xgmi_probe in the JSON; 0: skip)")
    ap.add_argument("--fp32-steps", type=int, default=5,
                    help="timed steps of each fp32 pass (default split convs, exact; 0: skip)")
    ap.add_argument("--amp-steps", type=int, default=10,
                    help="timed steps of the fp16 AMP-DDP pass (resnet_ddp_apex.py config; 0: skip)")
    ap.add_argument("--dp-steps", type=int, default=10,
                    help="timed steps of the DataParallel pass (resnet_dp.py config: rank 0 drives "
                         "all N GPUs in one process; 0: skip)")
    ap.add_argument("--util-steps", type=int, default=3,
                    help="untimed steps profiled for the device-busy %% when sysfs is unavailable")
    ap.add_argument("--nccl-channels", type=int, default=0,
                    help="RCCL channel count (NCCL_MIN_NCHANNELS = NCCL_MAX_NCHANNELS); 0: RCCL's "
                         "own tuning for the topology")
    ap.add_argument("--nccl-proto", default="", help="NCCL_PROTO (LL, LL128, Simple; '' = RCCL's choice)")
    ap.add_argument("--nccl-algo", default="", help="NCCL_ALGO (Ring, Tree; '' = RCCL's choice)")
    ap.add_argument("--rehearse-fold", action="store_true",
                    help="allow more ranks than visible GPUs (several ranks share a device: launch "
                         "rehearsals only, never a measurement)")
    return ap.parse_args()


def _launch_ranks(args) -> int | None:
    """``--gpus N`` means N ranks, however bench.py is started (the reference's DDP script spawns its
    own ranks, /root/reference/restnet_ddp.py:153-155). Started by a launcher (``WORLD_SIZE`` set),
    this process is one rank and the world must equal ``--gpus``. Started bare with ``--gpus N > 1``,
    this process becomes the launcher: it checks -- from sysfs, no HIP call -- that N GPUs are
    visible, starts ``torch.distributed.run`` with N ranks as a CHILD process (never an exec: the
    child ranks own the GPUs) on a 127.0.0.1 rendezvous, lets rank 0's single JSON line through on
    the shared stdout, and returns the launcher's exit code (non-zero when any rank failed).
    Returns None when this process should run the benchmark itself."""
    world_env = os.environ.get("WORLD_SIZE")
    if args.dp:
        return None     # one process driving --gpus devices (resnet_dp.py), never N ranks
    if world_env is not None:
        world = int(world_env)
        if world != args.gpus:
            print(f"bench: WORLD_SIZE {world} but --gpus {args.gpus}: the record would mislabel the "
                  f"run; pass --gpus {world}", file=sys.stderr, flush=True)
            return 2
        return None
    if args.gpus <= 1:
        return None
    if args.device == "cuda" and not args.rehearse_fold:
        from pytorch_distributed_amd.launch import visible_gpu_count
        n = visible_gpu_count()
        if n < args.gpus:
            print(f"bench: --gpus {args.gpus} needs {args.gpus} visible GPUs, this process sees {n} "
                  f"(--rehearse-fold shares devices for launch rehearsals)", file=sys.stderr, flush=True)
            return 2
    import signal
    import subprocess
    from pytorch_distributed_amd.launch import free_port
    env = dict(os.environ)
    env["PDA_BENCH_LAUNCHER"] = "self"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.abspath(__file__), *sys.argv[1:]]
    child = subprocess.Popen(cmd, env=env, start_new_session=True)

    def _forward(sig, _frame):
        # a timeout of the parent must also end every rank: the launcher stops its ranks (each in
        # a session of its own) on SIGTERM / SIGINT
        try:
            os.killpg(child.pid, sig)
        except OSError:
            pass
    for s in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(s, _forward)
    try:
        rc = child.wait()
    finally:
        if child.poll() is None:
            _forward(signal.SIGTERM, None)
            try:
                child.wait(timeout=30)
            except subprocess.TimeoutExpired:
                _forward(signal.SIGKILL, None)
    return rc if rc >= 0 else 128 - rc


def _configure_process(args) -> dict:
    """Everything that must precede the first HIP call of the process: the IPC mode HSA reads at
    its initialisation, the RCCL knobs a communicator reads at creation, and the NUMA binding (HIP's
    runtime threads inherit the affinity the process has when they start). Returns the effective
    RCCL/HSA settings for the JSON record."""
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    os.environ.setdefault("MX_WATCHDOG", "0")   # timed runs: no polling thread beside the step
    graph = getattr(args, "graph", -1)
    if getattr(args, "dp", False) or graph == 1 or (graph < 0 and GRAPH_DEFAULT):
        # graph replay needs the single-queue graph launch, set before HIP starts
        # (pytorch_distributed_amd/runtime/graphs.py GRAPH_QUEUES_VAR)
        os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "1")
    if args.nccl_channels > 0:
        os.environ["NCCL_MIN_NCHANNELS"] = os.environ["NCCL_MAX_NCHANNELS"] = str(args.nccl_channels)
    if args.nccl_proto:
        os.environ["NCCL_PROTO"] = args.nccl_proto
    if args.nccl_algo:
        os.environ["NCCL_ALGO"] = args.nccl_algo
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    numa = False
    if world > 1 and args.device == "cuda" and os.environ.get("PDA_BIND_NUMA", "1") != "0":
        # one rank per GPU, pinned to that GPU's NUMA node as the reference's
        # hfai.multiprocessing.spawn(bind_numa=True); the GPU count comes from the
        # KFD topology in sysfs, so no HIP call precedes the binding
        # (tests/test_bench_cpu.py::test_numa_binding_precedes_any_hip_call)
        from pytorch_distributed_amd.launch import bind_numa, visible_gpu_count
        numa = bind_numa(local_rank % max(visible_gpu_count(), 1))
    env = {k: v for k, v in sorted(os.environ.items())
           if k.startswith(("NCCL_", "RCCL_", "HSA_ENABLE_IPC", "GPU_MAX_HW_QUEUES"))}
    return {"comm_env": env, "numa_bound": numa}


class Ctx:
    def __init__(self, args):
        self.args = args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.cuda = args.device == "cuda"
        if self.cuda:
            ndev = max(torch.cuda.device_count(), 1)
            lws = int(os.environ.get("LOCAL_WORLD_SIZE", str(self.world)))
            if lws > ndev and not args.rehearse_fold and not args.dp:
                raise SystemExit(f"bench: {lws} ranks on this node but {ndev} visible GPU(s); "
                                 f"--rehearse-fold shares devices for launch rehearsals")
            self.device = torch.device("cuda", self.local_rank % ndev)  # >1 rank/GPU: rehearsals only
            torch.cuda.set_device(self.device)
        else:
            ndev = 1
            self.device = torch.device("cpu")
        self.ndev = ndev
        self.multi = self.world > 1 and not args.dp
        self.spread = {}

    def sync(self):
        if self.cuda:
            if self.args.dp:
                for d in range(self.args.gpus):
                    torch.cuda.synchronize(d)
            else:
                torch.cuda.synchronize(self.device)

    # host-side collectives on the gloo host group: the only RCCL communicator of the process is
    # the gradient communicator of the model (launch.host_group)
    def barrier(self):
        if self.multi:
            import torch.distributed as dist
            from pytorch_distributed_amd.launch import host_group
            self.sync()
            dist.barrier(group=host_group())
        self.sync()

    def allreduce(self, vals, op: str = "max"):
        import torch.distributed as dist
        from pytorch_distributed_amd.launch import host_group
        t = torch.tensor(vals, dtype=torch.float64)
        dist.all_reduce(t, op={"max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
                               "sum": dist.ReduceOp.SUM}[op], group=host_group())
        return t

    def allreduce_max(self, x: float) -> float:
        if not self.multi:
            return x
        return float(self.allreduce([x], "max")[0])


def _timed(ctx: Ctx, tr, first: int, steps: int, key: str = "headline") -> float:
    """``steps`` timed steps between barrier + device sync on both sides; returns the MAX elapsed
    over ranks and keeps the per-rank spread (min, max) in ``ctx.spread[key]`` so a straggler rank
    shows up in the record."""
    ctx.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        tr.step(first + i)
    ctx.barrier()
    el = time.perf_counter() - t0
    if not ctx.multi:
        ctx.spread[key] = (el, el)
        return el
    lo, hi = (float(v) for v in ctx.allreduce([-el, el], "max"))
    ctx.spread[key] = (-lo, hi)
    return hi


def _spread_record(ctx: Ctx) -> dict:
    """Per-rank timed-region spread of every timed pass: min / max seconds over ranks and the
    max-over-min excess in percent (0 on one rank)."""
    out = {}
    for k, (lo, hi) in ctx.spread.items():
        out[k] = {"min_s": round(lo, 4), "max_s": round(hi, 4),
                  "spread_pct": round(100.0 * (hi - lo) / lo, 2) if lo > 0 else None}
    return {"rank_time_spread": out}


def _diagnostics(ctx: Ctx, tr, first: int) -> dict:
    """N>1, after the timed region: bucket plan, RCCL world, exposed communication."""
    out = {"comm": None, "rccl_world": None, "buckets": None, "bucket_bytes": None,
           "exposed_comm_ms": None, "bucket_allreduce_ms": None}
    net = getattr(tr, "net", None)
    red = getattr(net, "reducer", None)
    if net is None or red is None:
        return out
    out["comm"] = type(net.comm).__name__
    out["rccl_world"] = getattr(net, "rccl_world", None)
    if getattr(red, "buckets", None):
        out["buckets"] = len(red.buckets)
        out["bucket_bytes"] = red.bucket_bytes
    nat = getattr(red, "native", None)
    if nat is not None and ctx.args.diag_steps > 0:
        exp, per = [], []
        nat.set_timing(True)
        for i in range(ctx.args.diag_steps):
            tr.step(first + i)
            ctx.sync()
            e, b = nat.timing()
            exp.append(e)
            per.append(b)
        nat.set_timing(False)
        out["exposed_comm_ms"] = round(statistics.median(exp), 4)
        out["bucket_allreduce_ms"] = [round(statistics.median(c), 4) for c in zip(*per)]
    return out


PROBE_BYTES = (16 << 10, 256 << 10, 2 << 20, 8 << 20, 32 << 20)


def _comm_probe(ctx: Ctx, tr) -> dict:
    """N>1, after the timed region: f32 all-reduce time of the communicator the gradient buckets
    use (the native RCCL one on GPU), at sizes spanning the bucket plan, so the xGMI cost model
    behind the bucket caps (parallel/reducer.py: T(S) = alpha + 2(n-1)/n S / busbw, alpha and
    eta assumed) is measured on the node the driver runs: alpha = T(16 KiB), bus bandwidth and
    eta = busbw / (7 x 153 GB/s) from T(32 MiB). Wall clock around REPS back-to-back calls with
    a device sync on both sides, ranks aligned by a barrier; the MAX over ranks."""
    net = getattr(tr, "net", None)
    comm = getattr(net, "comm", None)
    if comm is None or not ctx.args.comm_probe:
        return {}
    import torch.distributed as dist
    from pytorch_distributed_amd.launch import host_group
    n = ctx.world
    ms = []
    for b in PROBE_BYTES:
        t = torch.zeros(b // 4, device=ctx.device)
        reps = 20 if b <= (2 << 20) else 8
        for _ in range(3):
            comm.all_reduce(t)
        ctx.sync()
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            comm.all_reduce(t)
        ctx.sync()
        ms.append(1000.0 * (time.perf_counter() - t0) / reps)
        del t
    worst = torch.tensor(ms, dtype=torch.float64)
    dist.all_reduce(worst, op=dist.ReduceOp.MAX, group=host_group())
    ms = [round(float(v), 4) for v in worst]
    big = PROBE_BYTES[-1]
    busbw = 2.0 * (n - 1) / n * big / (ms[-1] * 1e-3) / 1e9
    return {"xgmi_probe": {"comm": type(comm).__name__, "bytes": list(PROBE_BYTES), "ms": ms,
                           "alpha_us": round(1000.0 * ms[0], 1),
                           "busbw_GBs": round(busbw, 1),
                           "eta_vs_7x153GBs": round(busbw / (7 * 153.0), 3)}}


def _verify_consistent(ctx: Ctx, tr) -> dict:
    """Bit-exact parameter + momentum checksum, MIN/MAX over ranks (N>1)."""
    cs = tr.state_checksum()
    perturb = os.environ.get("PDA_BENCH_PERTURB_RANK")
    if perturb is not None and int(perturb) == ctx.rank:
        cs = cs + 1
    if not ctx.multi:
        return {"weights_consistent": None, "checksum": [int(v) for v in cs.tolist()]}
    import torch.distributed as dist
    from pytorch_distributed_amd.launch import host_group
    lo, hi = cs.cpu().clone(), cs.cpu().clone()     # int64: exact on the gloo host group
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=host_group())
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=host_group())
    ok = bool(torch.equal(lo, hi))
    return {"weights_consistent": ok, "checksum": [int(v) for v in cs.tolist()]}


def _fp32_pass(ctx: Ctx, args, mode: str = "split") -> dict:
    """Short fp32 pass (reference precision), each rank locally (no all-reduce). ``mode``: the f32
    convolution math of the native engine -- "split" (the fp32 default: bf16 MFMA on a hi/lo
    three-term split, ~16 significant bits per product, at or below the error of the TF32
    convolutions the reference's fp32 runs use by default on A100 -- tests/test_f32_precision_gpu.py)
    keyed ``fp32_*``, or "exact" (MFMA 16x16x4 f32, f32 rounding only) keyed ``fp32_exact_*``."""
    from pytorch_distributed_amd.bench_step import make_trainer
    from pytorch_distributed_amd.ops import native_ops as K
    old, K._F32_CONV = K._F32_CONV, mode
    try:
        tr = make_trainer(args.arch, args.batch, torch.float32, ctx.device, engine=args.engine,
                          world=1, rank=0, bucket_mb=args.bucket_mb, image_size=args.image_size)
        if mode != "exact" and tr.engine != "native":
            return {}
        for i in range(2):
            tr.step(i)
        key = "fp32" if mode == "split" else "fp32_exact"
        el = _timed(ctx, tr, 2, args.fp32_steps, key)
    finally:
        K._F32_CONV = old
    world = ctx.world if ctx.multi else 1
    res = {f"{key}_images_per_sec": round(args.batch * world * args.fp32_steps / el, 2),
           f"{key}_ms_per_step": round(1000.0 * el / args.fp32_steps, 3)}
    if mode == "split":
        res.update({"fp32_engine": tr.engine, "fp32_conv": "split (bf16 MFMA hi/lo, >= TF32)",
                    "fp32_conv_note": "fp32_* = split convs (per-conv error <= TF32, "
                                      "tests/test_f32_precision_gpu.py); fp32_exact_* = f32 MFMA. "
                                      "TF32 is torch's cudnn.allow_tf32 default, which the reference "
                                      "never changes; its GPU model is not stated, so whether its "
                                      "fp32 bar ran TF32 is parity unpinned",
                    "fp32_mode": "single" if world == 1 else "per-rank local steps, no all-reduce"})
    del tr
    if ctx.cuda:
        torch.cuda.empty_cache()
    return res


def _gather_util(ctx: Ctx, mine):
    """Average GPU busy % over the ranks' devices (the reference's "Avg GPU Util" panel)."""
    if not ctx.multi:
        return mine
    t = ctx.allreduce([mine if mine is not None else 0.0, 1.0 if mine is not None else 0.0], "sum")
    return round(float(t[0] / t[1]), 1) if t[1] > 0 else None


def _all_ranks(ctx: Ctx, flag: bool) -> bool:
    """True iff ``flag`` holds on every rank (a decision that gates collective work)."""
    if not ctx.multi:
        return flag
    return bool(ctx.allreduce([1.0 if flag else 0.0], "min")[0] > 0)


def _guarded(ctx: Ctx, name: str, fn, *a) -> dict:
    """A secondary pass must not cost the headline record: its failure is reported in the JSON
    (``<name>_error``) on every rank, and the ranks stay in step (the pass ends on a barrier)."""
    try:
        return fn(*a)
    except Exception as e:   # noqa: BLE001
        traceback.print_exc()
        return {f"{name}_error": f"{type(e).__name__}: {e}"[:300]}


def _amp_pass(ctx: Ctx, args) -> dict:
    """The resnet_ddp_apex.py configuration (/root/reference/resnet_ddp_apex.py:27-34,107): fp16
    compute with dynamic loss scaling (native LossScaler: device-side inf scan + scale update, no
    host sync), DDP gradient all-reduce over RCCL, fp32 master weights. Timed like the headline;
    then the bit-exact cross-rank checksum of parameters + momentum."""
    from pytorch_distributed_amd.bench_step import make_trainer
    if ctx.cuda:
        torch.cuda.reset_peak_memory_stats(ctx.device)
    tr = make_trainer(args.arch, args.batch, torch.float16, ctx.device, engine=args.engine,
                      world=ctx.world, rank=ctx.rank, bucket_mb=args.bucket_mb,
                      image_size=args.image_size)
    for i in range(3):
        tr.step(i)
    with BusySampler([ctx.device.index] if ctx.cuda else []) as busy:
        el = _timed(ctx, tr, 3, args.amp_steps, "amp_fp16")
    amp_util = busy.overall()
    if not _all_ranks(ctx, amp_util is not None) and ctx.cuda and args.util_steps > 0:
        kb = kernel_busy(lambda i: tr.step(1000 + i), args.util_steps, [ctx.device.index])
        amp_util = kb.get(ctx.device.index)
    cons = _verify_consistent(ctx, tr)
    world = ctx.world if ctx.multi else 1
    sc = getattr(tr, "scaler", None)
    res = {"amp_fp16_images_per_sec": round(args.batch * world * args.amp_steps / el, 2),
           "amp_fp16_ms_per_step": round(1000.0 * el / args.amp_steps, 3),
           "amp_config": f"fp16 + dynamic loss scaling, {'DDP over RCCL' if ctx.multi else 'single GPU'}"
                         f" ({tr.engine}; resnet_ddp_apex.py)",
           "amp_dtype": "fp16",
           "amp_weights_consistent": cons.get("weights_consistent"),
           "amp_loss": tr.last_loss(),
           "amp_loss_scale": float(sc.get_scale()) if sc is not None and hasattr(sc, "get_scale") else None,
           "amp_max_mem_gb": round(torch.cuda.max_memory_allocated(ctx.device) / 1e9, 2) if ctx.cuda else None,
           "amp_gpu_util_pct": _gather_util(ctx, amp_util)}
    base = BASELINE.get(world)
    if base:
        res["amp_vs_baseline"] = round(res["amp_fp16_images_per_sec"] / base, 3)
        # the reference's "Apex" bar is fp16 autocast AMP too: like for like
        res["amp_vs_baseline_precision"] = "fp16 AMP vs the reference's fp16 AMP (Apex) bar"
    del tr
    if ctx.cuda:
        torch.cuda.empty_cache()
    return res


def _dp_pass(ctx: Ctx, args, dtype) -> dict:
    """The resnet_dp.py configuration (/root/reference/resnet_dp.py:82): ONE process drives all N
    GPUs (global batch 400 x N). Rank 0 runs it as a child process (``bench.py --dp --gpus N``:
    persistent native replicas, per-replica graph-replayed forward/backward, in-process grouped
    RCCL all-reduce, replicated fused SGD, replicas checked bit-identical) under a time limit, while
    the other ranks wait on the TCP store -- a host-side wait (an RCCL barrier would occupy their
    GPUs), and a failure or hang of the pass costs its keys, never the headline record."""
    import subprocess
    n = min(ctx.world if ctx.multi else 1, torch.cuda.device_count()) if ctx.cuda else 1
    store = None
    if ctx.multi:
        import torch.distributed as dist
        store = dist.distributed_c10d._get_default_store()
    limit = float(os.environ.get("PDA_BENCH_DP_TIMEOUT_S", "420"))
    res = {}
    if ctx.rank == 0:
        try:
            env = {k: v for k, v in os.environ.items()
                   if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                                "ROLE_RANK", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
                   and not k.startswith("TORCHELASTIC")}
            cmd = [sys.executable, os.path.abspath(__file__), "--dp", "--gpus", str(n),
                   "--steps", str(args.dp_steps), "--warmup", "3", "--batch", str(args.batch),
                   "--arch", args.arch, "--image-size", str(args.image_size), "--dtype", args.dtype,
                   "--fp32-steps", "0", "--amp-steps", "0", "--dp-steps", "0",
                   "--device", "cuda" if ctx.cuda else "cpu"]
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=limit)
            lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
            if r.returncode != 0 or not lines:
                res = {"dp_error": f"rc={r.returncode}: {r.stderr.strip()[-300:]}"}
            else:
                rec = json.loads(lines[-1])
                res = {"dp_images_per_sec": rec["value"], "dp_ms_per_step": rec["ms_per_step"],
                       "dp_config": f"{rec['config']['parallelism']}: one process, {n} GPU(s), global "
                                    f"batch {rec['config']['global_batch']}, {rec['config']['engine']}, "
                                    f"{rec['dtype']} (resnet_dp.py)",
                       "dp_dtype": rec.get("dtype"),
                       "dp_vs_baseline_precision": rec.get("vs_baseline_precision"),
                       "dp_replicas_consistent": rec.get("replicas_consistent"),
                       "dp_loss": rec.get("loss"), "dp_max_mem_gb": rec.get("max_mem_gb"),
                       "dp_gpu_util_pct": rec.get("gpu_util_pct"), "dp_vs_baseline": rec.get("vs_baseline"),
                       "dp_exposed_comm_ms": rec.get("exposed_comm_ms"),
                       "dp_segments": rec.get("dp_segments"),
                       "dp_replay_ms_per_step": rec.get("dp_replay_ms_per_step"),
                       "dp_replay_vs_eager": rec.get("dp_replay_vs_eager"),
                       "dp_replay_segments": rec.get("dp_replay_segments"),
                       "dp_side_graphs": rec.get("dp_side_graphs")}
        except subprocess.TimeoutExpired:
            res = {"dp_error": f"timeout after {limit:.0f} s"}
        finally:
            if store is not None:
                store.set("pda_bench_dp_done", json.dumps(res))
    elif store is not None:
        store.wait(["pda_bench_dp_done"], datetime.timedelta(seconds=limit + 120))
        res = json.loads(store.get("pda_bench_dp_done").decode())
    return res


def main():
    args = parse()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    rc = _launch_ranks(args)           # before any HIP call of this process
    if rc is not None:
        sys.stdout.flush()
        sys.stderr.flush()
        sys.exit(rc)
    proc = _configure_process(args)    # before Ctx: Ctx initialises HIP (set_device)
    proc["launcher"] = ("bench.py -> torch.distributed.run (self-launched ranks)"
                        if os.environ.get("PDA_BENCH_LAUNCHER") == "self"
                        else "external launcher" if "WORLD_SIZE" in os.environ else "single process")
    ctx = Ctx(args)
    if ctx.world > 1:
        import torch.distributed as dist
        timeout = datetime.timedelta(seconds=float(os.environ.get("PDA_DIST_TIMEOUT_S", "600")))
        backend = os.environ.get("PDA_DIST_BACKEND", "nccl" if ctx.cuda else "gloo")
        os.environ.setdefault("PDA_RCCL_INIT_TIMEOUT_S", str(timeout.total_seconds()))
        # no device_id: torch's NCCL communicator stays uncreated; gradients go through the
        # model's own RCCL communicator, host-side values through the gloo host group
        dist.init_process_group(backend, timeout=timeout)
        from pytorch_distributed_amd.launch import host_group
        host_group()

    from pytorch_distributed_amd.bench_step import make_trainer
    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.dtype]
    graph = args.graph == 1 or (args.graph < 0 and ctx.world == 1 and GRAPH_DEFAULT)
    world = ctx.world
    if args.dp:
        if ctx.world > 1:
            raise SystemExit("--dp is one process driving --gpus devices; do not launch it with torchrun")
        from pytorch_distributed_amd.bench_step import make_dp_trainer
        tr = make_dp_trainer(args.arch, args.batch, dtype, args.gpus, args.image_size,
                             device=args.device)
        world = args.gpus            # images/sec over all devices of the process
    else:
        tr = make_trainer(args.arch, args.batch, dtype, ctx.device, engine=args.engine,
                          world=ctx.world, rank=ctx.rank, bucket_mb=args.bucket_mb,
                          image_size=args.image_size, graph=graph)

    for i in range(args.warmup):
        tr.step(i)
    ctx.sync()
    util_devs = (list(range(args.gpus)) if args.dp else [ctx.device.index]) if ctx.cuda else []
    with BusySampler(util_devs) as busy:
        elapsed = _timed(ctx, tr, args.warmup, args.steps)   # barrier + sync on both sides, MAX
    loss = tr.last_loss()
    nxt = args.warmup + args.steps
    diag = _diagnostics(ctx, tr, nxt) if ctx.multi else {}
    if ctx.multi:
        diag.update(_comm_probe(ctx, tr))
    if args.dp and getattr(tr.dp, "replicas", None):
        # one more (untimed) step with HIP events at the end of backward and after the last
        # gradient all-reduce (per-stage slices overlapped with the backward's later segments)
        tr.dp.timing = True
        tr.step(nxt)
        for d in tr.dp.device_ids:
            torch.cuda.synchronize(d)
        tr.dp.timing = False
        ex = tr.dp.exposed_comm_ms()
        diag["exposed_comm_ms"] = None if ex is None else round(ex, 4)
        rg = tr.dp._graphs[0]
        diag["dp_segments"] = len(rg.graphs)
        diag["dp_side_graphs"] = sum(g is not None for g in getattr(rg, "sides", []))
        nxt += 1
    if args.dp and not getattr(tr.dp, "replicas", None) and ctx.cuda and args.steps > 0:
        # one device: the eager step above is what torch's DataParallel does for one device; the
        # replica-graph replay an N > 1 run takes (per-block segment graphs + weight-gradient side
        # graphs) is timed here too, so that path has a number on every 1-GPU record
        tr.dp.force_replay = True
        nw = 1 + max(2, args.warmup)  # the capture step, then as many warm replays as the headline
        for i in range(nw):
            tr.step(nxt + i)
        rel = _timed(ctx, tr, nxt + nw, args.steps, "dp_replay")
        nxt += nw + args.steps
        diag["dp_replay_ms_per_step"] = round(1000.0 * rel / args.steps, 3)
        diag["dp_replay_vs_eager"] = round(rel / elapsed, 4)
        diag["dp_replay_segments"] = len(tr.dp._graphs[0].graphs)
        diag["dp_side_graphs"] = sum(g is not None for g in getattr(tr.dp._graphs[0], "sides", []))
        tr.dp.force_replay = False
    if args.dp:   # every replica must hold bit-identical weights (the replicated fused SGD)
        try:
            tr.state_checksum()
            consistency = {"replicas_consistent": True}
        except RuntimeError:
            consistency = {"replicas_consistent": False}
    else:
        consistency = _verify_consistent(ctx, tr) if hasattr(tr, "state_checksum") else {}
    ms = 1000.0 * elapsed / max(args.steps, 1)
    value = args.batch * world * args.steps / elapsed
    # the reference's bars are ResNet-50 on GPUs: no ratio for other models or the CPU config
    base = ((BASELINE_DP if args.dp else BASELINE).get(world)
            if args.arch == "resnet50" and ctx.cuda else None)
    cfg = {"model": args.arch, "global_batch": args.batch * world,
           "per_gpu_batch": args.batch, "seq_len": None,
           "parallelism": (f"dataparallel{world}" if args.dp else f"dp{world}"),
           "engine": tr.engine,
           "hip_graph": bool(getattr(tr, "graphed", None)),
           "optimizer": "SGD(lr=0.1, momentum=0.9, wd=1e-4)",
           "bucket_cap_mb": args.bucket_mb if ctx.multi else None}
    max_mem = round(torch.cuda.max_memory_allocated(ctx.device) / 1e9, 2) if ctx.cuda else None
    mine = busy.overall()
    util_method = "sysfs gpu_busy_percent" if mine is not None else None
    if not _all_ranks(ctx, mine is not None) and ctx.cuda and args.util_steps > 0:
        # no sysfs counter (on some rank): the kernels' own records, on every rank alike
        kb = kernel_busy(lambda i: tr.step(nxt + 100 + i), args.util_steps, util_devs)
        v = [x for x in kb.values() if x is not None]
        mine = round(sum(v) / len(v), 1) if v else None
        util_method = f"kernel-interval union over {args.util_steps} untimed steps (torch.profiler)"
    util = _gather_util(ctx, mine)
    extra = {}
    if not args.dp:
        del tr
        if ctx.cuda:
            torch.cuda.empty_cache()
        if args.fp32_steps > 0 and args.dtype != "fp32":
            extra.update(_fp32_pass(ctx, args))
            extra.update(_fp32_pass(ctx, args, "exact"))
        if args.amp_steps > 0 and args.dtype != "fp16":
            extra.update(_guarded(ctx, "amp_fp16", _amp_pass, ctx, args))
        if args.dp_steps > 0:   # (on the CPU: the launch / store hand-off rehearsal)
            extra.update(_guarded(ctx, "dp", _dp_pass, ctx, args, dtype))
    if ctx.rank == 0:
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
            "vs_baseline_precision": (f"{args.dtype} (this run) vs the reference's fp32/TF32 bar"
                                      if args.dtype != "fp32" else "fp32 vs fp32/TF32"),
            "dtype": args.dtype,
            "data": (f"synthetic ({'on-device' if ctx.cuda else 'host'} generated 3x{args.image_size}x"
                     f"{args.image_size}, random-init weights)"),
            "config": cfg,
            "loss": loss,
            "max_mem_gb": max_mem,
            "gpu_util_pct": util,
            "gpu_util_method": util_method,
            **proc, **diag, **consistency, **extra,
        }
        rec.update(_spread_record(ctx))
        if extra.get("fp32_images_per_sec") and base:
            rec["vs_baseline_fp32"] = round(extra["fp32_images_per_sec"] / base, 3)
            if "fp32_split_images_per_sec" in extra:
                rec["vs_baseline_fp32_split"] = round(extra["fp32_split_images_per_sec"] / base, 3)
        print(json.dumps(rec), flush=True)
    if consistency.get("weights_consistent") is False:
        print(f"bench: rank {ctx.rank}: parameters differ across ranks after training "
              f"(checksum {consistency['checksum']})", file=sys.stderr, flush=True)
        sys.stderr.flush()
        os._exit(3)
    bad = [k for k in ("amp_weights_consistent", "dp_replicas_consistent") if extra.get(k) is False]
    if consistency.get("replicas_consistent") is False:
        bad.append("replicas_consistent")
    if bad:
        print(f"bench: rank {ctx.rank}: inconsistent state after a secondary pass: {bad}",
              file=sys.stderr, flush=True)
        os._exit(3)
    if ctx.multi:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    try:
        main()
    except SystemExit:
        raise
    except BaseException:
        # a failed rank must not hang in teardown (stuck collective threads): report and leave
        traceback.print_exc()
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(1)
