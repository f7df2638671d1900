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
        red.native.close()
        comm.close()
    finally:
        dist.destroy_process_group()
