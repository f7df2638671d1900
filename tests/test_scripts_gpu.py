"""T6 tier on the GPU: the entrypoints run the native engine end to end (tiny epochs), including
preemption -> resume through latest.pt and the fp16 loss-scaled ("Apex") script."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    e = dict(os.environ)
    e.update({"MX_ARCH": "resnet50", "MX_EPOCHS": "2", "MX_STEPS_PER_EPOCH": "3", "MX_VAL_STEPS": "2",
              "MX_BATCH": "16", "MX_IMAGE_SIZE": "64", "PYTHONPATH": ROOT, "MASTER_IP": "127.0.0.1",
              "MX_NPROCS": "1", "MX_LR": "0.01", "MX_METRICS": "1"})
    e.update(kw)
    return e


def _run(script, tmp_path, **kw):
    r = subprocess.run([sys.executable, os.path.join(ROOT, script)], cwd=tmp_path, env=_env(**kw),
                       capture_output=True, text=True, timeout=600)
    return r


@pytest.mark.parametrize("script,outdir", [("resnet_single_gpu.py", "resnet_single"),
                                           ("restnet_ddp.py", "resnet_ddp"),
                                           ("resnet_ddp_apex.py", "resnet_ddp_amp"),
                                           ("resnet_dp.py", "resnet_dp")])
def test_entrypoint_native(tmp_path, script, outdir):
    r = _run(script, tmp_path, MASTER_PORT=str(29600 + hash(script) % 200))
    assert r.returncode == 0, r.stderr[-4000:]
    assert "Epoch: 1, Loss: " in r.stdout and "cost time per epoch: " in r.stdout
    m = (tmp_path / "output" / outdir / "metrics.jsonl").read_text()
    assert '"engine": "native"' in m
    if script == "resnet_ddp_apex.py":
        assert "float16" in m
    # the reference's three report panels per epoch: time, avg GPU util, GPU memory
    import json
    for line in m.strip().splitlines():
        rec = json.loads(line)
        assert rec["epoch_s"] > 0 and rec["gpu_mem_gb"] > 0
        assert rec["gpu_util_pct"] is not None and 0 < rec["gpu_util_pct"] <= 100, rec


def test_suspend_resume_native(tmp_path):
    from pytorch_distributed_amd.utils.suspend import REQUEUE_EXIT_CODE
    r = _run("resnet_ddp_apex.py", tmp_path, MX_SUSPEND_AT_STEP="2", MASTER_PORT="29811")
    assert r.returncode == REQUEUE_EXIT_CODE, r.stderr[-4000:]
    ck = torch.load(tmp_path / "output/resnet_ddp_amp/latest.pt", weights_only=True)
    assert ck["step"] == 2 and "scaler" in ck and ck["scaler"]["scale"] > 0
    assert len(ck["optimizer"]["state"]) == 161
    r = _run("resnet_ddp_apex.py", tmp_path, MASTER_PORT="29812")
    assert r.returncode == 0, r.stderr[-4000:]
    assert "resume: epoch 0 step 2" in r.stdout


def test_entrypoint_native_exact_fp32(tmp_path):
    """MX_DTYPE=fp32 (the reference scripts' own precision) runs on the native engine too."""
    r = _run("resnet_single_gpu.py", tmp_path, MX_DTYPE="fp32")
    assert r.returncode == 0, r.stderr[-4000:]
    m = (tmp_path / "output" / "resnet_single" / "metrics.jsonl").read_text()
    assert '"engine": "native"' in m and "float32" in m


def test_native_resume_from_reference_format_checkpoint(tmp_path):
    """A latest.pt in the reference's format (plain torch ResNet-50 / SGD / StepLR state_dicts,
    OIHW weights, per-parameter momentum buffers) resumes on the native engine."""
    from pytorch_distributed_amd.models import build_model
    torch.manual_seed(0)
    model = build_model("resnet50")
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=30, gamma=0.1)
    torch.nn.functional.cross_entropy(model(torch.randn(2, 3, 64, 64)),
                                      torch.tensor([1, 2])).backward()
    opt.step()
    out = tmp_path / "output" / "resnet_single"
    out.mkdir(parents=True)
    torch.save({"model": model.state_dict(), "optimizer": opt.state_dict(),
                "scheduler": sched.state_dict(), "acc": 0.5, "epoch": 1, "step": 1},
               out / "latest.pt")
    r = _run("resnet_single_gpu.py", tmp_path, MX_LOG_EVERY="1")
    assert r.returncode == 0, r.stderr[-4000:]
    assert "resume: epoch 1 step 1 (best acc 0.5)" in r.stdout
    assert "epoch: 1, step: 1" in r.stdout and "epoch: 1, step: 0" not in r.stdout


def test_single_gpu_graph_mode_matches_eager(tmp_path):
    """MX_GRAPH=1: resnet_single_gpu.py replays each training step from ONE HIP graph (captured on
    the first step, re-captured when StepLR changes the LR); the validation losses it prints are
    bit-identical to the eager run's."""
    def losses(sub, **kw):
        d = tmp_path / sub
        d.mkdir()
        r = _run("resnet_single_gpu.py", d, MX_DTYPE="bf16", **kw)
        assert r.returncode == 0, r.stderr[-4000:]
        return [l for l in r.stdout.splitlines() if l.startswith("Epoch: ")]
    eager, graph = losses("eager", MX_GRAPH="0"), losses("graph", MX_GRAPH="1")
    assert len(eager) == 2 and eager == graph, (eager, graph)
