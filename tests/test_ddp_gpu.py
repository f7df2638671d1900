"""T5 tier on a single MI355X: the native DDP path with 2 ranks sharing one GPU over gloo
(RCCL refuses two ranks on one device), plus the native RCCL communicator at world size 1."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["PDA_COMM"] = "torch"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", world_size=world, rank=rank)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from pytorch_distributed_amd.data import SyntheticImageNet
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    from pytorch_distributed_amd.parallel import DistributedDataParallel
    torch.manual_seed(0)
    ref = build_model("resnet18")
    local = NativeResNet(build_model("resnet18"), device=dev, image_size=64)
    local.load_state_dict(ref.state_dict())
    model = NativeResNet(ref, device=dev, image_size=64)
    if rank == 1:  # perturb: the DDP constructor must broadcast rank 0's weights
        with torch.no_grad():
            model.flat_params.add_(0.5)
    ddp = DistributedDataParallel(model, bucket_cap_mb=4.0)
    gen = model.input_generator(SyntheticImageNet("train", image_size=64))
    x, y = gen(torch.arange(8) + 8 * rank)
    crit = model.make_criterion()
    opt = model.make_optimizer(lr=0.05)
    opt.zero_grad()
    crit(ddp(x), y).backward()
    torch.cuda.synchronize()
    g_ddp = model.flat_grad.clone()
    # local gradient of the same batch without DDP, averaged across ranks by hand
    lcrit = local.make_criterion()
    local.zero_grad_flat()
    lcrit(local(x), y).backward()
    g_loc = local.flat_grad.clone()
    dist.all_reduce(g_loc)
    g_loc /= world
    err = ((g_ddp - g_loc).norm() / g_loc.norm()).item()
    opt.step()
    torch.cuda.synchronize()
    p = model.flat_params.clone()
    pl = [torch.empty_like(p) for _ in range(world)]
    dist.all_gather(pl, p)
    same = all(torch.equal(pl[0], t) for t in pl)
    q.put((rank, err, same))
    dist.destroy_process_group()


def test_native_ddp_two_ranks_one_gpu():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    for rank, err, same in res:
        assert err < 1e-5, (rank, err)
        assert same


def test_rccl_communicator_world1():
    if dist.is_initialized():
        pytest.skip("process group already initialised")
    port = _port()
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", world_size=1, rank=0,
                            device_id=dev)
    try:
        from pytorch_distributed_amd.parallel.rccl import RcclCommunicator
        c = RcclCommunicator(dev)
        c.start_watchdog(0.05)
        t = torch.arange(1000, dtype=torch.float32, device=dev)
        h = c.all_reduce_async(t)
        c.wait(c.all_reduce_async(t, op="avg"))
        c.wait(h)
        c.broadcast(t, 0)
        c.barrier()
        c.check()
        torch.cuda.synchronize()
        assert torch.equal(t, torch.arange(1000, dtype=torch.float32, device=dev))
        c.close()
    finally:
        dist.destroy_process_group()


def test_native_ddp_cpp_reducer_world1():
    """DDP over the native RCCL communicator: the C++ bucket reducer (csrc/comm/reducer.cpp)
    launches every bucket once per step, ordered after both backward streams, and the averaged
    gradient at world size 1 equals the local gradient bit for bit."""
    if dist.is_initialized():
        pytest.skip("process group already initialised")
    port = _port()
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", world_size=1, rank=0,
                            device_id=dev)
    try:
        from pytorch_distributed_amd.data import SyntheticImageNet
        from pytorch_distributed_amd.models import build_model
        from pytorch_distributed_amd.models.native import NativeResNet
        from pytorch_distributed_amd.parallel import DistributedDataParallel
        from pytorch_distributed_amd.parallel.rccl import RcclCommunicator
        torch.manual_seed(0)
        ref = build_model("resnet50")
        local = NativeResNet(build_model("resnet50"), device=dev, image_size=64)
        local.load_state_dict(ref.state_dict())
        model = NativeResNet(ref, device=dev, image_size=64)
        comm = RcclCommunicator(dev)
        ddp = DistributedDataParallel(model, bucket_cap_mb=8.0, comm=comm)
        red = ddp.reducer
        assert red.native is not None, "C++ reducer not in use"
        nb = len(red.buckets)
        assert nb >= 3
        gen = model.input_generator(SyntheticImageNet("train", image_size=64))
        crit, lcrit = model.make_criterion(), local.make_criterion()
        for step in range(2):
            x, y = gen(torch.arange(8) + 8 * step)
            model.zero_grad_flat()
            crit(ddp(x), y).backward()
            local.zero_grad_flat()
            lcrit(local(x), y).backward()
            torch.cuda.synchronize()
            assert red.native.launched == nb * (step + 1)
            assert torch.equal(model.flat_grad, local.flat_grad)
        # bucket boundaries sit on the xGMI quantum (8 ranks x 7 links x 256 B)
        from pytorch_distributed_amd.models.native import BUCKET_QUANTUM
        assert all(s % BUCKET_QUANTUM == 0 and e % BUCKET_QUANTUM == 0 for s, e in red.buckets)
        assert ddp.rccl_world == 1
        # timing diagnostics (bench.py exposed_comm_ms / bucket_allreduce_ms)
        red.native.set_timing(True)
        x, y = gen(torch.arange(8) + 64)
        model.zero_grad_flat()
        crit(ddp(x), y).backward()
        torch.cuda.synchronize()
        exposed, per = red.native.timing()
        red.native.set_timing(False)
        assert exposed >= 0.0 and len(per) == nb and all(v >= 0.0 for v in per), (exposed, per)
        red.native.close()
        comm.close()
    finally:
        dist.destroy_process_group()


def test_rccl_abort_world1_reducer_raises_cleanly():
    """Failure handling: after an abort (what the watchdog does on an async error)
    the bucket reducer's launches raise CommAbortedError instead of touching a freed
    communicator, and the communicator / reducer can then be closed in either order."""
    if dist.is_initialized():
        pytest.skip("process group already initialised")
    port = _port()
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", world_size=1, rank=0,
                            device_id=dev)
    try:
        from pytorch_distributed_amd.parallel.rccl import CommAbortedError, RcclCommunicator
        for close_comm_first in (True, False):
            comm = RcclCommunicator(dev)
            assert comm.rccl_count == 1 and not comm.aborted
            flat = torch.ones(4 * 3584, device=dev)
            red = comm.make_bucket_reducer(flat, [(0, 3584), (3584, 4 * 3584)])
            red.ready(3584)
            red.finish()
            torch.cuda.synchronize()
            assert torch.equal(flat, torch.ones_like(flat))      # avg over 1 rank
            comm.abort()
            assert comm.aborted
            with pytest.raises(CommAbortedError):
                red.ready(3584)
            with pytest.raises(CommAbortedError):
                red.finish()
            with pytest.raises(CommAbortedError):
                comm.all_reduce(flat)
            with pytest.raises(CommAbortedError):
                comm.check()
            if close_comm_first:
                comm.close()
                red.close()
            else:
                red.close()
                comm.close()
            with pytest.raises(CommAbortedError):
                red.ready(1)
            with pytest.raises(CommAbortedError):
                comm.broadcast(flat)
    finally:
        dist.destroy_process_group()


def _syncbn_worker(rank, world, port, q):
    os.environ["PDA_COMM"] = "torch"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", world_size=world, rank=rank)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from pytorch_distributed_amd.data import SyntheticImageNet
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    from pytorch_distributed_amd.parallel import DistributedDataParallel, convert_sync_batchnorm
    torch.manual_seed(0)
    sd = {k: v.clone() for k, v in build_model("resnet18").state_dict().items()}
    f32 = torch.float32
    nets = []
    for _ in range(3):
        m = NativeResNet(build_model("resnet18"), device=dev, dtype=f32, image_size=64)
        m.load_state_dict(sd)
        nets.append(m)
    model, full, half = convert_sync_batchnorm(nets[0]), nets[1], nets[2]
    assert torch.equal(model.flat_params, full.flat_params)
    ddp = DistributedDataParallel(model, bucket_cap_mb=4.0)
    assert ddp.bn_comm is not None
    gen = model.input_generator(SyntheticImageNet("train", image_size=64))
    x, y = gen(torch.arange(8) + 8 * rank)
    xf, yf = gen(torch.arange(16))
    model.zero_grad_flat()
    model.make_criterion()(ddp(x), y).backward()
    torch.cuda.synchronize()
    g_sync = model.flat_grad.clone()
    # the same 16 images in ONE process: what SyncBN over 2 x 8 must reproduce
    full.zero_grad_flat()
    full.make_criterion()(full(xf), yf).backward()
    g_full = full.flat_grad.clone()
    # per-rank statistics (no SyncBN), gradients averaged by hand: must differ
    half.zero_grad_flat()
    half.make_criterion()(half(x), y).backward()
    g_half = half.flat_grad.clone()
    dist.all_reduce(g_half)
    g_half /= world
    torch.cuda.synchronize()
    nf = g_full.norm()
    err_sync = ((g_sync - g_full).norm() / nf).item()
    err_half = ((g_half - g_full).norm() / nf).item()
    err_rm = ((model.flat_buffers - full.flat_buffers).norm() / full.flat_buffers.norm()).item()
    segs = []   # per-block gradient error (diagnostics)
    prev = 0
    for b in model.block_bounds:
        if b > prev:
            d = g_full[prev:b]
            segs.append(round(((g_sync[prev:b] - d).norm() / (d.norm() + 1e-30)).item(), 6))
            prev = b
    q.put((rank, err_sync, err_half, err_rm, segs))
    dist.destroy_process_group()


def test_native_ddp_sync_batchnorm_two_ranks():
    """SyncBatchNorm (MX_SYNC_BN / convert_sync_batchnorm) on the native engine: 2 ranks x 8
    images give the gradients and running statistics of one 16-image batch (exact fp32 path;
    tools/diag_syncbn.py also checks both against a torch fp32 oracle)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_syncbn_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    # exact fp32 with f64 statistics totals all-reduced before the finalize: measured 1.8e-6 (round
    # 2; per-rank statistics are off by 1.23). A ReLU input within rounding of 0 could still flip
    # its recomputed mask between the 8- and the 16-image runs (~1e-3 on one layer), hence 1e-4.
    for rank, err_sync, err_half, err_rm, segs in res:
        print(f"rank {rank}: SyncBN grad error {err_sync:.2e} (per-rank BN {err_half:.2e})")
        assert err_sync < 1e-4, (rank, err_sync, err_half, err_rm, segs)
        assert err_half > 20 * err_sync, (rank, err_sync, err_half)
        assert err_rm < 1e-5, (rank, err_rm)


def test_ddp_step_costs_no_more_than_bare_step(tmp_path):
    """Each rank's DDP step (native RCCL communicator, C++ bucket reducer, torch's own NCCL
    communicator NOT created -- the bench / trainer configuration) must cost about what the bare
    native step costs. A high-priority comm stream made it +13-15 ms (28.8 -> 43.3 ms per
    ResNet-50 step at GPU_MAX_HW_QUEUES=4; profiles/ddp_overhead_r3.md): checked in a fresh process
    so no earlier HIP stream or communicator changes the queue mapping."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "ddp_sync_diag.py"), "--steps", "8",
                        "--port", str(_port())], capture_output=True, text=True, timeout=300,
                       env={**os.environ, "PYTHONPATH": root})
    assert r.returncode == 0, r.stderr[-3000:]
    res = {l.split(" ", 1)[0]: json.loads(l.split(" ", 1)[1]) for l in r.stdout.splitlines()
           if l.startswith(("bare_", "ddp_"))}
    bare, ddp = res["bare_nosync"]["ms"], res["ddp_nosync"]["ms"]
    # the ratio itself is a measurement (printed; profiles/ddp_overhead_r3.md records +0.5 %); the
    # assertion only guards the regression it targets (+13-15 ms/step), so a shared or loaded box
    # cannot fail it with no code change
    print(f"DDP step {ddp:.2f} ms vs bare {bare:.2f} ms ({100.0 * (ddp / bare - 1.0):+.1f} %)")
    assert ddp < bare + 8.0, res
