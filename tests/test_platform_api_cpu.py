"""A script written against the reference's ``hfai`` platform API ports by changing its imports.

``_main`` follows the structure of the reference's DDP script (env rendezvous, spawn with NUMA
binding, ``hfai.nccl.distributed`` init, ``hfai.nn.parallel.DistributedDataParallel``,
``hfai.datasets.ImageNet(...).loader(...)`` with a DistributedSampler, suspend polling, validate
with ``dist.reduce``) -- here on CPU (gloo), ResNet-18, tiny images, 2 ranks."""
import os

import torch

import pytorch_distributed_amd.platform as hfai
import pytorch_distributed_amd.platform.nccl.distributed as dist
from pytorch_distributed_amd.data import DistributedSampler
from pytorch_distributed_amd.models import build_model
from pytorch_distributed_amd.platform.nn.parallel import DistributedDataParallel


def _main(local_rank, out_dir):
    ip, port = os.environ["MASTER_IP"], os.environ["MASTER_PORT"]
    hosts, rank = 1, 0                                # WORLD_SIZE / RANK (nodes) of the reference
    gpus = 2
    dist.init_process_group(backend="nccl", init_method=f"tcp://{ip}:{port}",
                            world_size=hosts * gpus, rank=rank * gpus + local_rank)
    torch.manual_seed(0)
    model = DistributedDataParallel(build_model("resnet18", 10))
    train_ds = hfai.datasets.ImageNet("train", image_size=32, num_samples=64)
    sampler = DistributedSampler(train_ds, dist.get_world_size(), dist.get_rank(), shuffle=True)
    loader = train_ds.loader(8, sampler=sampler, num_workers=4, pin_memory=True)
    crit = torch.nn.CrossEntropyLoss()
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    sampler.set_epoch(0)
    model.train()
    for step, (x, y) in enumerate(loader):
        if step == 2:
            break
        loss = crit(model(x), y % 10)
        opt.zero_grad()
        loss.backward()
        opt.step()
        assert not hfai.client.receive_suspend_command()
    val = hfai.datasets.ImageNet("val", image_size=32, num_samples=16)
    model.eval()
    stats = torch.zeros(2)
    with torch.no_grad():
        for x, y in val.loader(8, sampler=DistributedSampler(val, dist.get_world_size(), dist.get_rank())):
            stats[0] += (model(x).argmax(-1) == (y % 10)).sum()
            stats[1] += x.shape[0]
    dist.reduce(stats, 0)
    flat = torch.cat([p.detach().flatten() for p in model.module.parameters()])
    ref = flat.clone()
    dist.broadcast(ref, 0)
    same = bool(torch.equal(flat, ref))
    if dist.get_rank() == 0:
        with open(os.path.join(out_dir, "result.txt"), "w") as f:
            f.write(f"{same} {int(stats[1].item())}")
    dist.destroy_process_group()


def test_reference_style_script_on_platform_api(tmp_path, monkeypatch):
    monkeypatch.setenv("MASTER_IP", "127.0.0.1")
    monkeypatch.delenv("MASTER_PORT", raising=False)
    monkeypatch.setenv("MX_DATA", "synthetic")
    hfai.multiprocessing.spawn(_main, args=(str(tmp_path),), nprocs=2, bind_numa=True)
    same, total = (tmp_path / "result.txt").read_text().split()
    assert same == "True"          # DDP kept the replicas identical
    assert int(total) == 16        # validation counters reduced across both ranks


def test_bind_numa_respects_allowed_cpus():
    """bind_numa never widens the CPU set and is a no-op without KFD topology (CPU boxes)."""
    import os
    from pytorch_distributed_amd.launch import bind_numa
    before = os.sched_getaffinity(0)
    changed = bind_numa(0)
    after = os.sched_getaffinity(0)
    assert isinstance(changed, bool)
    assert after <= before and after
    if not changed:
        assert after == before
    os.sched_setaffinity(0, before)


def test_nccl_shim_uses_the_framework_communicator(monkeypatch):
    """Once DDP has registered the process's device communicator, ``hfai.nccl.distributed``'s
    reduce / all_reduce / broadcast on that device go through it (no second communicator); a
    ``group`` argument or an op it lacks goes to torch."""
    from pytorch_distributed_amd.parallel import comm as C
    calls = []

    class Fake:
        def reduce(self, t, dst, op):
            calls.append(("reduce", dst, op))

        def all_reduce(self, t, op="sum"):
            calls.append(("all_reduce", op))

        def broadcast(self, t, src=0):
            calls.append(("broadcast", src))

    monkeypatch.setattr(C, "_DEFAULTS", {})
    C.register_default(Fake(), torch.device("cpu"))
    x = torch.zeros(4)
    dist.reduce(x, 0)
    dist.all_reduce(x, op=dist.ReduceOp.MAX)
    assert dist.broadcast(x, 1, async_op=True).wait()
    assert calls == [("reduce", 0, "sum"), ("all_reduce", "max"), ("broadcast", 1)]
    torch_calls = []
    monkeypatch.setattr(torch.distributed, "all_reduce",
                        lambda t, op=None, group=None, async_op=False: torch_calls.append(op))
    dist.all_reduce(x, op=dist.ReduceOp.PRODUCT)          # not a native op -> torch
    dist.all_reduce(x, group=object())                     # explicit group -> torch
    assert len(torch_calls) == 2 and len(calls) == 3
