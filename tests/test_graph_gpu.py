"""HIP-graph capture of the native training step: replaying the captured step must reproduce the
eager step bit for bit (every kernel is deterministic -- no float atomics), for bf16 and for the
fp16 AMP path (device-side loss scaling), and an LR change must trigger a re-capture."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(dtype, graph, steps=4, lr_change_at=None):
    from pytorch_distributed_amd.models.native import NativeTrainer
    dev = torch.device("cuda", 0)
    tr = NativeTrainer("resnet50", 16, dtype, dev, image_size=64, graph=graph)
    losses = []
    for i in range(steps):
        if lr_change_at is not None and i == lr_change_at:
            tr.opt.param_groups[0]["lr"] = 0.01
        tr.step(i)
        losses.append(tr.last_loss())
    torch.cuda.synchronize()
    return tr, losses


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_graph_replay_matches_eager(dtype):
    te, le = _run(dtype, graph=False)
    tg, lg = _run(dtype, graph=True)
    assert tg.graphed.captures == 1
    assert le == lg, (le, lg)
    assert torch.equal(te.model.flat_params, tg.model.flat_params)
    assert torch.equal(te.opt.flat_mom, tg.opt.flat_mom)
    assert torch.equal(te.model.flat_buffers, tg.model.flat_buffers)   # BN running stats
    if dtype == torch.float16:
        assert te.scaler.get_scale() == tg.scaler.get_scale()


def test_graph_recaptures_on_lr_change():
    te, le = _run(torch.bfloat16, graph=False, steps=4, lr_change_at=2)
    tg, lg = _run(torch.bfloat16, graph=True, steps=4, lr_change_at=2)
    assert tg.graphed.captures == 2
    assert le == lg
    assert torch.equal(te.model.flat_params, tg.model.flat_params)


@pytest.mark.parametrize("mode", ["block", "stage"])
def test_wgrad_fork_granularity_is_bitwise_neutral(mode, monkeypatch):
    """The weight-gradient stream's fork granularity (per conv / per block / per stage; the graph
    capture uses "stage" for the duration of the capture only) changes no value."""
    te, le = _run(torch.bfloat16, graph=False, steps=3)
    monkeypatch.setenv("PDA_WGRAD_BATCH", mode)
    tb, lb = _run(torch.bfloat16, graph=False, steps=3)
    assert tb.model._wbatch_mode == mode
    assert le == lb
    assert torch.equal(te.model.flat_params, tb.model.flat_params)
    assert torch.equal(te.opt.flat_mom, tb.opt.flat_mom)


def test_graph_schedule_is_scoped_to_the_capture():
    tg, _ = _run(torch.bfloat16, graph=True, steps=2)
    assert tg.graphed.captures == 1
    assert tg.model._wbatch_mode == "0"      # eager steps after the capture keep their schedule


def test_capture_refuses_priority_streams():
    """hipStreamEndCapture segfaults when a captured stream has a non-default priority (ROCm 7:
    profiles/ab_r3_dma.md section 5, faulthandler trace at torch.cuda.graphs capture_end); the
    capture refuses such a stream with an error instead."""
    from pytorch_distributed_amd.models.native import NativeTrainer
    tr = NativeTrainer("resnet18", 8, torch.bfloat16, torch.device("cuda", 0), image_size=64, graph=True)
    tr.model._side = torch.cuda.Stream(torch.device("cuda", 0), priority=-1)
    with pytest.raises(RuntimeError, match="priority"):
        tr.step(0)


def test_graph_capture_with_two_hw_queues(tmp_path):
    """Capture + replay with fewer hardware queues than streams (GPU_MAX_HW_QUEUES=2: the main, the
    weight-gradient and the capture side stream share queues) in a fresh process."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GPU_MAX_HW_QUEUES="2", PDA_NO_BUILD="1")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--graph", "1", "--steps", "2",
                        "--warmup", "2", "--batch", "32", "--image-size", "64", "--fp32-steps", "0",
                        "--amp-steps", "0", "--dp-steps", "0"], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert rec["config"]["hip_graph"] is True and rec["value"] > 0
