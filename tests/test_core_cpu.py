"""T0/T1 tier: pure-Python components with torch CPU oracles."""
import math
import os

import pytest
import torch
from torch import nn

from pytorch_distributed_amd.config import config_for
from pytorch_distributed_amd.data import DistributedSampler, SyntheticImageNet, synthetic_images
from pytorch_distributed_amd.models import resnet18, resnet50
from pytorch_distributed_amd.parallel.reducer import plan_buckets
from pytorch_distributed_amd.utils.checkpoint import load_latest, save_best, save_latest


def test_config_defaults_match_reference():
    s = config_for("single", env={})
    assert (s.epochs, s.batch_size, s.num_workers, s.lr, s.momentum, s.weight_decay) == \
        (100, 400, 4, 0.1, 0.9, 1e-4)
    assert s.save_path == "output/resnet_single"
    assert config_for("dp", env={}).batch_size == 3200
    assert config_for("ddp", env={}).save_path == "output/resnet_ddp"
    a = config_for("ddp_amp", env={})
    assert a.save_path == "output/resnet_ddp_amp" and a.dtype == "fp16"
    o = config_for("single", env={"MX_EPOCHS": "3", "MX_DTYPE": "bf16"})
    assert o.epochs == 3 and o.dtype == "bf16"
    with pytest.raises(ValueError):
        config_for("single", env={"MX_DTYPE": "int8"})


def test_cli_flags_mirror_env():
    # no flags -> identical to env-only; flags override env
    assert config_for("single", env={}, argv=[]) == config_for("single", env={})
    c = config_for("ddp", env={"MX_EPOCHS": "3"},
                   argv=["--epochs", "5", "--steps-per-epoch", "7", "--dtype", "bf16"])
    assert (c.epochs, c.steps_per_epoch, c.dtype) == (5, 7, "bf16")
    with pytest.raises(SystemExit):
        config_for("single", env={}, argv=["--no-such-flag", "1"])


def test_resnet50_census_matches_torchvision():
    m = resnet50()
    n = sum(p.numel() for p in m.parameters())
    assert n == 25_557_032                      # SURVEY §2.7 model census
    assert len(list(m.parameters())) == 161
    assert len(list(m.buffers())) == 159
    sd = m.state_dict()
    for k in ["conv1.weight", "bn1.running_mean", "layer1.0.downsample.0.weight",
              "layer4.2.bn3.num_batches_tracked", "fc.weight", "fc.bias", "layer2.3.conv2.weight"]:
        assert k in sd
    assert sd["layer2.0.conv2.weight"].shape == (128, 128, 3, 3)
    # v1.5: stride on the 3x3 conv
    assert m.layer2[0].conv2.stride == (2, 2) and m.layer2[0].conv1.stride == (1, 1)
    # kaiming fan_out init: std = sqrt(2 / (cout*k*k))
    w = m.layer3[0].conv2.weight
    assert abs(w.std().item() - math.sqrt(2.0 / (256 * 9))) < 0.01 * math.sqrt(2.0 / (256 * 9)) * 10
    assert torch.all(m.bn1.weight == 1) and torch.all(m.bn1.bias == 0)


def test_resnet18_forward_backward_cpu():
    m = resnet18(num_classes=10)
    x = torch.randn(2, 3, 64, 64)
    y = m(x)
    assert y.shape == (2, 10)
    y.sum().backward()
    assert m.conv1.weight.grad is not None


def test_sampler_matches_torch():
    from torch.utils.data.distributed import DistributedSampler as TorchDS
    ds = list(range(103))
    for world in (1, 2, 4, 8):
        for rank in range(world):
            for epoch in (0, 3):
                a = DistributedSampler(ds, world, rank, shuffle=True, seed=7)
                b = TorchDS(ds, world, rank, shuffle=True, seed=7)
                a.set_epoch(epoch)
                b.set_epoch(epoch)
                assert list(a) == list(b)
                assert len(a) == len(b)


def test_synthetic_deterministic_and_learnable():
    ids = torch.tensor([0, 5, 17, 5])
    x1, y1 = synthetic_images(ids, 0, "train", 1000, 32)
    x2, y2 = synthetic_images(ids, 0, "train", 1000, 32)
    assert torch.equal(x1, x2) and torch.equal(y1, y2)
    assert torch.equal(x1[1], x1[3])
    assert not torch.equal(x1[0], x1[1])
    xv, _ = synthetic_images(ids, 0, "val", 1000, 32)
    assert not torch.equal(xv, x1)
    assert x1.shape == (4, 3, 32, 32) and y1.dtype == torch.int64
    assert 0 <= int(y1.min()) and int(y1.max()) < 1000
    ds = SyntheticImageNet("train", 1000, 0, 10, 16)
    xs, ys = ds.batch(torch.arange(200))
    # class tint makes channel means label-dependent
    m0 = xs[ys == ys[0]][:, 0].mean()
    assert len(ds) == 1000 and torch.isfinite(m0)


def test_loader_len_and_resume_seek():
    ds = SyntheticImageNet("train", 1003, 0, 10, 8)
    ld = ds.loader(100)
    assert len(ld) == 11
    all_b = [b for b in ld]
    assert all_b[-1][0].shape[0] == 3
    rest = [b for _, b in ld.iter_from(4)]
    assert len(rest) == 7 and torch.equal(rest[0][1], all_b[4][1])


def test_plan_buckets():
    MiB = 1 << 20
    g = plan_buckets([MiB // 2, MiB // 2, MiB, 20 * MiB, 20 * MiB, 3 * MiB, MiB], 32 * MiB, MiB,
                     2 * MiB)
    assert g[0] == [0, 1]
    flat = [i for b in g for i in b]
    assert flat == list(range(7))
    assert sum([MiB // 2, MiB // 2, MiB, 20 * MiB, 20 * MiB, 3 * MiB, MiB][i] for i in g[-1]) <= 2 * MiB


def test_checkpoint_schema(tmp_path):
    m = resnet18(num_classes=10)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    sch = torch.optim.lr_scheduler.StepLR(opt, 30, 0.1)
    m(torch.randn(2, 3, 32, 32)).sum().backward()
    opt.step()
    save_latest(tmp_path, m.state_dict(), opt.state_dict(), sch.state_dict(), 0.5, 3, 17,
                scaler_sd={"scale": 1024.0})
    ck = load_latest(tmp_path)
    assert set(ck) == {"model", "optimizer", "scheduler", "acc", "epoch", "step", "scaler"}
    assert ck["epoch"] == 3 and ck["step"] == 17
    m2 = resnet18(num_classes=10)
    m2.load_state_dict(ck["model"])
    for a, b in zip(m.state_dict().values(), m2.state_dict().values()):
        assert torch.equal(a, b)
    save_best(tmp_path, m.state_dict())
    assert (tmp_path / "best.pt").exists()
    assert load_latest(tmp_path / "nothing") is None


def test_suspend_monitor_step_trigger(monkeypatch):
    from pytorch_distributed_amd.utils.suspend import SuspendMonitor
    mon = SuspendMonitor(signals=(), at_step=3)
    hits = []
    for _ in range(5):
        mon.tick()
        hits.append(mon.requested())
    assert hits == [False, False, True, True, True]


def test_suspend_monitor_sentinel(tmp_path):
    from pytorch_distributed_amd.utils.suspend import SuspendMonitor
    f = tmp_path / "stop"
    mon = SuspendMonitor(signals=(), sentinel=str(f))
    assert not mon.requested()
    f.write_text("")
    assert mon.requested()


def test_loss_scaler_state_machine_matches_gradscaler():
    from pytorch_distributed_amd.amp import LossScaler
    p = nn.Parameter(torch.ones(4))
    opt = torch.optim.SGD([p], lr=0.1)
    s = LossScaler(init_scale=8.0, growth_interval=2)
    scales = []
    for step in range(6):
        loss = (p * 2).sum()
        s.scale(loss).backward()
        if step == 3:
            p.grad[0] = float("inf")
        before = p.detach().clone()
        s.step(opt)
        if step == 3:
            assert torch.equal(before, p.detach())      # skipped
        s.update()
        opt.zero_grad()
        scales.append(s.get_scale())
    assert scales == [8.0, 16.0, 16.0, 8.0, 8.0, 16.0]
    sd = s.state_dict()
    s2 = LossScaler()
    s2.load_state_dict(sd)
    assert s2.get_scale() == 16.0


def test_f32_conv_mode_dtype_and_tile_mapping(monkeypatch):
    """MX_F32_CONV / PDA_F32_CONV: f32 tensors map to kernel dtype 0 (exact f32 MFMA) or 3
    (split bf16 MFMA); the split kernels exist only as single-stage tiles of at most 128 x 128, so
    every (bm, bn) request is mapped onto one of those; 16-bit tensors are never affected."""
    import torch
    from pytorch_distributed_amd.ops import native_ops as K
    f32, bf16 = torch.zeros(1), torch.zeros(1, dtype=torch.bfloat16)
    monkeypatch.setattr(K, "_F32_CONV", "exact")
    assert K._kdt(f32) == 0 and K._kdt(bf16) == 1
    monkeypatch.setattr(K, "_F32_CONV", "split")
    assert K._kdt(f32) == 3 and K._kdt(bf16) == 1
    assert K._ktile(128, 128, 3) == (-128, 128)
    assert K._ktile(-256, 128, 3) == (-128, 128)
    assert K._ktile(64, 64, 3) == (-64, 64)
    assert K._ktile(128, 256, 3) == (-128, 128)
    assert K._ktile(128, 64, 1) == (128, 64)          # other dtypes untouched


def test_stream_cfg_is_fixed():
    """The BN apply streaming policy (csrc/bn.hip StreamCfg) is the measured one, no env knob."""
    from pytorch_distributed_amd.ops import ext
    assert ext.stream_cfg() == (-1, 3, 65536, 50)


def test_loss_scaler_refuses_second_fused_step():
    """The fused native step (inf scan + scale update in one kernel) moves the scale inside
    step(); a second optimizer stepped before update() would unscale by the updated scale, so the
    scaler refuses it (GradScaler updates once per iteration)."""
    from pytorch_distributed_amd.amp import LossScaler

    class FusedOpt:
        param_groups = []

        def __init__(self):
            self.calls = 0

        def step_amp(self, *a):
            self.calls += 1

    s = LossScaler(init_scale=8.0)
    s.scale(torch.ones(1))
    o1, o2 = FusedOpt(), FusedOpt()
    s.step(o1)
    with pytest.raises(RuntimeError, match="twice"):
        s.step(o2)
    s.update()
    s.step(o2)                      # a new iteration is fine
    assert o1.calls == 1 and o2.calls == 1


def test_lds_dma_tile_codes_and_fallback():
    """Tile codes of the conv launches: 1000 + rows = LDS-DMA 8-wave tile, 2000 + rows = its
    tap-reuse (HALO) form; they exist for 16-bit operands without the BN prologue only, and any
    other launch is mapped onto the register-staged 128-row tile."""
    from pytorch_distributed_amd.ops import native_ops as K
    assert K.tile_rows(1256) == 256 and K.tile_rows(2256) == 256 and K.tile_rows(-128) == 128
    assert K._ktile(1256, 128, 1) == (1256, 128) and K._ktile(2256, 128, 2) == (2256, 128)
    assert K._ktile(1128, 256, 0) == (-128, 128)            # f32: no DMA kernels
    assert K._ktile(2256, 128, 1, pro=True) == (-128, 128)  # prologue needs register staging
    g = K.ConvGeom(400, 14, 14, 256, 256, 3, 3, 1, 1)
    assert K.fwd_tile(g, 400, torch.bfloat16) == (2256, 128)
    assert K.fwd_tile(g, 400, torch.bfloat16, pro=True)[0] < 1000
    assert K.fwd_tile(g, 400, torch.float32)[0] < 1000
    # data gradients: the HALO tile for 3x3 stride-1 (PDA_DGRAD_HALO), register-staged otherwise
    assert K.dgrad_tile(g, 400) == ((2256, 128) if K._DGRAD_HALO else K.dgrad_tile(g, 400, dma=False))
    assert K.dgrad_tile(g, 400, dma=False)[0] < 1000
    g1 = K.ConvGeom(400, 14, 14, 256, 1024, 1, 1, 1, 0)
    assert K.dgrad_tile(g1, 400)[0] < 1000
    assert K.dgrad_slabs(g, 400, dtype=torch.float32) == math.ceil(400 * 196 / K.tile_rows(
        K.dgrad_tile(g, 400, dma=False)[0]))


def test_dedicated_conv_kernel_routing(monkeypatch):
    """Which convs conv_fwd hands to the dedicated stem kernel: the space-to-depth stem geometry to
    csrc/stem.hip (16-bit, H % 4, W % 16, W <= 128); statistics tiles of one output row."""
    from pytorch_distributed_amd.ops import native_ops as K

    class Lib:
        pda_stem_fwd = object()
    monkeypatch.setattr(K.ext, "lib", lambda: Lib)
    g = K.stem_s2d_geom(400, 224)
    assert K.stem_fwd_ok(g, torch.bfloat16) and K.stem_fwd_ok(g, torch.float16)
    assert not K.stem_fwd_ok(g, torch.float32)
    assert not K.stem_fwd_ok(K.stem_s2d_geom(2, 40), torch.bfloat16)    # W = 20: not % 16
    assert not K.stem_fwd_ok(K.stem_s2d_geom(2, 288), torch.bfloat16)   # W = 144 > 128
    assert K.stem_stats_rows(g) == 112


def test_dataparallel_segment_bounds_and_step_busy(monkeypatch):
    """DataParallel's graph-split policy (PDA_DP_SEGMENTS: stage bounds of a native module, none
    for a single device or mode 0, a clear error otherwise) and the HIP-event busy fallback of the
    epoch metrics (no device: no value, never a made-up one)."""
    from pytorch_distributed_amd.parallel.dp import DataParallel
    from pytorch_distributed_amd.utils.gpu_util import StepBusy

    class Fake:
        def stage_bounds(self):
            return [100, 200, 300]

    dp = DataParallel.__new__(DataParallel)     # no devices here: only the policy's inputs
    dp.__dict__.update(module=Fake(), replicas=[object()])
    monkeypatch.setenv("PDA_DP_SEGMENTS", "stage")
    assert dp._segment_bounds() == [100, 200, 300]
    monkeypatch.setenv("PDA_DP_SEGMENTS", "0")
    assert dp._segment_bounds() == []
    monkeypatch.setenv("PDA_DP_SEGMENTS", "stage")
    dp.__dict__["replicas"] = []
    assert dp._segment_bounds() == []
    monkeypatch.setenv("PDA_DP_SEGMENTS", "block")
    with pytest.raises(ValueError):
        dp._segment_bounds()
    with StepBusy(None) as sb:
        sb.begin()
        sb.end()
    assert sb.overall() is None
