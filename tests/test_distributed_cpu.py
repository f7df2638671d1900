"""T4 tier: DDP / reducer logic on CPU with gloo, world 2."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mlp():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(16, 64), nn.ReLU(), nn.Linear(64, 64), nn.Tanh(),
                         nn.Linear(64, 10))


def _ddp_worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", world_size=world,
                            rank=rank)
    from pytorch_distributed_amd.parallel import DistributedDataParallel
    torch.manual_seed(1 + rank)  # different init per rank -> ctor broadcast must fix it
    m = _mlp()
    if rank == 1:
        with torch.no_grad():
            for p in m.parameters():
                p.add_(1.0)
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.001)  # tiny buckets -> several buckets
    g = torch.Generator().manual_seed(123)
    x = torch.randn(8, 16, generator=g)
    y = torch.randint(0, 10, (8,), generator=g)
    xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
    opt = torch.optim.SGD(ddp.parameters(), lr=0.1, momentum=0.9)
    for it in range(2):
        opt.zero_grad()
        nn.functional.cross_entropy(ddp(xs), ys).backward()
        grads = [p.grad.clone() for p in m.parameters()]
        opt.step()
    q.put((rank, [g.numpy() for g in grads], [p.detach().clone().numpy() for p in m.parameters()]))
    dist.destroy_process_group()


def test_ddp_grads_equal_full_batch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (g, w)) for r, g, w in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    # reference: single process, full batch, same init as rank 0 (seed 1)
    torch.manual_seed(1)
    m = _mlp()
    g = torch.Generator().manual_seed(123)
    x = torch.randn(8, 16, generator=g)
    y = torch.randint(0, 10, (8,), generator=g)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    for it in range(2):
        opt.zero_grad()
        nn.functional.cross_entropy(m(x), y).backward()
        ref_g = [p.grad.clone() for p in m.parameters()]
        opt.step()
    for r in range(world):
        for a, b in zip(res[r][0], ref_g):
            torch.testing.assert_close(torch.from_numpy(a), b, rtol=1e-5, atol=1e-6)
        for a, b in zip(res[r][1], m.parameters()):
            torch.testing.assert_close(torch.from_numpy(a), b.detach(), rtol=1e-5, atol=1e-6)


def _suspend_worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", world_size=world,
                            rank=rank)
    from pytorch_distributed_amd.utils.suspend import SuspendMonitor
    mon = SuspendMonitor(signals=(), at_step=(3 if rank == 1 else None))
    out = []
    for _ in range(4):
        mon.tick()
        out.append(mon.requested())
    q.put((rank, out))
    dist.destroy_process_group()


def test_collective_suspend_decision():
    """Q5 fix: only rank 1 is asked, but every rank agrees at the same step."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_suspend_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
    assert res[0] == res[1] == [False, False, True, True]


def _env(tmp, **kw):
    e = dict(os.environ)
    e.update({"MX_ARCH": "resnet18", "MX_EPOCHS": "2", "MX_STEPS_PER_EPOCH": "2",
              "MX_VAL_STEPS": "1", "MX_BATCH": "4", "MX_IMAGE_SIZE": "32", "MX_NUM_CLASSES": "10",
              "MX_DEVICE": "cpu", "PYTHONPATH": ROOT, "MASTER_IP": "127.0.0.1",
              "MASTER_PORT": str(_port()), "OMP_NUM_THREADS": "2"})
    e.update(kw)
    return e


@pytest.mark.parametrize("script", ["resnet_single_gpu.py", "resnet_dp.py", "restnet_ddp.py",
                                    "resnet_ddp_apex.py"])
def test_cli_scripts_cpu(tmp_path, script):
    """T6: every entrypoint runs with no args; log lines match the reference formats."""
    env = _env(tmp_path, MX_NPROCS="2")
    r = subprocess.run([sys.executable, os.path.join(ROOT, script)], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = r.stdout
    assert "Epoch: 0, Loss: " in out and "Acc1: " in out and "Acc5: " in out
    assert "cost time per epoch: " in out
    name = {"resnet_single_gpu.py": "resnet_single", "resnet_dp.py": "resnet_dp",
            "restnet_ddp.py": "resnet_ddp", "resnet_ddp_apex.py": "resnet_ddp_amp"}[script]
    if script == "resnet_single_gpu.py":
        assert "epoch: 0, step: 0" in out
    if "New Best Acc" in out:
        assert (tmp_path / "output" / name / "best.pt").exists()


def test_suspend_resume_cli(tmp_path):
    """Fault injection: suspend at step 3, rerun resumes from latest.pt at the next step."""
    from pytorch_distributed_amd.utils.suspend import REQUEUE_EXIT_CODE
    env = _env(tmp_path, MX_SUSPEND_AT_STEP="3", MX_EPOCHS="2", MX_STEPS_PER_EPOCH="4",
               MX_LOG_EVERY="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "resnet_single_gpu.py")], cwd=tmp_path,
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == REQUEUE_EXIT_CODE, r.stderr[-3000:]
    ck = torch.load(tmp_path / "output/resnet_single/latest.pt", weights_only=True)
    assert ck["epoch"] == 0 and ck["step"] == 3
    env.pop("MX_SUSPEND_AT_STEP")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "resnet_single_gpu.py")], cwd=tmp_path,
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "resume: epoch 0 step 3" in r.stdout
    assert "epoch: 0, step: 3" in r.stdout and "epoch: 0, step: 2" not in r.stdout


def test_resume_from_reference_format_checkpoint(tmp_path):
    """Interop: a latest.pt written the way the reference writes it -- plain torch model / SGD /
    StepLR state_dicts of a torchvision-layout model (reference restnet_ddp.py:37-44) -- resumes in
    this framework's trainer; the final weights load back into the plain torch model."""
    from pytorch_distributed_amd.models import build_model
    torch.manual_seed(0)
    model = build_model("resnet18", 10)          # the CLI env below uses MX_NUM_CLASSES=10
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=30, gamma=0.1)
    x, y = torch.randn(4, 3, 32, 32), torch.randint(0, 10, (4,))
    nn.functional.cross_entropy(model(x), y).backward()
    opt.step()                                  # populates momentum buffers
    out = tmp_path / "output" / "resnet_single"
    out.mkdir(parents=True)
    torch.save({"model": model.state_dict(), "optimizer": opt.state_dict(),
                "scheduler": sched.state_dict(), "acc": 0.25, "epoch": 0, "step": 2},
               out / "latest.pt")
    env = _env(tmp_path, MX_EPOCHS="1", MX_STEPS_PER_EPOCH="4", MX_LOG_EVERY="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "resnet_single_gpu.py")], cwd=tmp_path,
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "resume: epoch 0 step 2 (best acc 0.25)" in r.stdout
    assert "epoch: 0, step: 2" in r.stdout and "epoch: 0, step: 1" not in r.stdout
    best = out / "best.pt"
    if best.exists():                           # written only if accuracy beat 0.25
        build_model("resnet18", 10).load_state_dict(torch.load(best, weights_only=True))


def test_convert_sync_batchnorm_keeps_state_dict_and_env_flag():
    """MX_SYNC_BN / convert_sync_batchnorm: a plain torch model gets nn.SyncBatchNorm layers with the
    torchvision state_dict keys unchanged (the native engine path is tested on the GPU:
    tests/test_ddp_gpu.py::test_native_ddp_sync_batchnorm_two_ranks); off by default."""
    from pytorch_distributed_amd.config import config_for
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.parallel import convert_sync_batchnorm
    m = build_model("resnet18", 10)
    keys = list(m.state_dict())
    s = convert_sync_batchnorm(m)
    assert list(s.state_dict()) == keys
    assert sum(isinstance(x, nn.SyncBatchNorm) for x in s.modules()) == 20
    assert not config_for("ddp", env={}).sync_bn
    assert config_for("ddp", env={"MX_SYNC_BN": "1"}).sync_bn
