"""Native DataParallel semantics on one GPU: two replicas sharing cuda:0 (plain-copy sync path)
must produce the same update as one model on the concatenated batch."""
import warnings

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_native_dataparallel_matches_single_model():
    from pytorch_distributed_amd.data import SyntheticImageNet
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    from pytorch_distributed_amd.parallel import DataParallel
    torch.manual_seed(0)
    ref = build_model("resnet18")
    sd = {k: v.clone() for k, v in ref.state_dict().items()}
    single = NativeResNet(ref, device=DEV, image_size=64)
    ref2 = build_model("resnet18")
    ref2.load_state_dict(sd)
    dp = DataParallel(NativeResNet(ref2, device=DEV, image_size=64), device_ids=[0, 0])
    gen = single.input_generator(SyntheticImageNet("train", image_size=64))
    x, y = gen(torch.arange(16))
    # BN statistics are per replica in DP (as in torch): compare against two half batches
    crit = torch.nn.CrossEntropyLoss()
    opt_dp = dp.make_optimizer(lr=0.05, momentum=0.9, weight_decay=1e-4)
    opt_dp.zero_grad()
    crit(dp(x), y).backward()
    torch.cuda.synchronize()
    g_dp = dp.module.flat_grad.clone()
    assert torch.equal(dp.module.flat_grad, dp.replicas[0].flat_grad)
    # reference: gradient of the mean loss over the global batch, each half with its own BN stats
    g_ref = torch.zeros_like(g_dp)
    for h in range(2):
        single.zero_grad_flat()
        out = single(x[h * 8:(h + 1) * 8])
        (crit(out, y[h * 8:(h + 1) * 8]) * 0.5).backward()
        g_ref += single.flat_grad
    err = ((g_dp - g_ref).norm() / g_ref.norm()).item()
    assert err < 1e-4, err
    opt_dp.step()
    torch.cuda.synchronize()
    assert torch.equal(dp.module.flat_params, dp.replicas[0].flat_params)


@pytest.mark.parametrize("side", ["conv", "1", "0"])
@pytest.mark.parametrize("segments", ["stage", "0"])
def test_native_dataparallel_graph_step_matches_eager(segments, side, monkeypatch):
    """train_step replayed from per-replica HIP graphs == the same schedule launched eagerly (bit
    for bit, 4 steps incl. SGD), and its first step == crit(dp(x), y).backward() (autograd DP with
    ATen's cross-entropy: equal up to the 16-bit rounding of dlogits). ``stage``: the completed
    gradient slice after layer4 / layer3 / layer2 is reduced on a comm stream while the next
    segments replay (4 reductions). ``side`` (PDA_DP_SIDE): the weight gradients are recorded as
    graphs of their own -- one per weight gradient ("conv", the main chain split where each one's
    inputs are complete) or one per residual block ("1") -- replayed on the second stream beside
    the following main-chain segment."""
    monkeypatch.setenv("PDA_DP_SEGMENTS", segments)
    monkeypatch.setenv("PDA_DP_SIDE", side)
    from pytorch_distributed_amd.data import SyntheticImageNet
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    from pytorch_distributed_amd.parallel import DataParallel
    torch.manual_seed(0)
    sd = build_model("resnet18").state_dict()
    dps = []
    for _ in range(3):
        r = build_model("resnet18")
        r.load_state_dict(sd)
        dps.append(DataParallel(NativeResNet(r, device=DEV, image_size=64), device_ids=[0, 0]))
    auto, eager, graphed = dps
    assert graphed.graph_step_ok()
    gen = eager.module.input_generator(SyntheticImageNet("train", image_size=64))
    x, y = gen(torch.arange(16))
    crit = torch.nn.CrossEntropyLoss()
    oa = auto.make_optimizer(lr=0.05, momentum=0.9, weight_decay=1e-4)
    oa.zero_grad()
    la = crit(auto(x), y)
    la.backward()
    oe = eager.make_optimizer(lr=0.05, momentum=0.9, weight_decay=1e-4)
    og = graphed.make_optimizer(lr=0.05, momentum=0.9, weight_decay=1e-4)
    for step in range(4):
        x, y = gen(torch.arange(16) + 16 * step)
        graphed.timing = step == 3
        le = eager.train_step(x, y, oe, graph=False)
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            lg = graphed.train_step(x, y, og)
        # (conv mode: a block boundary right after a weight gradient's split records nothing)
        assert not [w for w in caught if "Graph is empty" in str(w.message)], step
        torch.cuda.synchronize()
        if step == 0:
            assert abs(la.item() - lg.item()) < 1e-4 * abs(la.item())
            err = ((auto.module.flat_grad - graphed.module.flat_grad).norm()
                   / auto.module.flat_grad.norm()).item()
            assert err < 2e-2, err
        assert le.item() == lg.item(), (step, le.item(), lg.item())
        assert torch.equal(eager.module.flat_grad, graphed.module.flat_grad), step
        assert torch.equal(eager.module.flat_params, graphed.module.flat_params), step
        assert torch.equal(graphed.module.flat_params, graphed.replicas[0].flat_params)
        assert torch.equal(eager.module.flat_buffers, graphed.module.flat_buffers)
    assert graphed._graphs[0].graph is not None and eager._graphs[0].graph is None
    rg = graphed._graphs[0]
    nblk = len(graphed.module.blocks)
    nside = sum(g is not None for g in rg.sides)
    if side == "conv":   # one side graph per weight gradient (every conv + the fc), after its segment
        # (the shortcut's weight gradient shares conv_n's side graph unless a tail fold's
        # bn_fold launch separates them)
        m = graphed.module
        nconv = sum(len(b.units) + (b.ds is not None and bool(m._tail_fold_ok(b, 8)))
                    for b in m.blocks) + 2
        assert nside == nconv and nconv <= len(rg.graphs) <= nconv + len(rg.splits) + 1, \
            (nside, nconv, len(rg.graphs))
    else:
        assert len(rg.graphs) == (nblk + 1 if side == "1" else (4 if segments == "stage" else 1))
        assert (nside > nblk // 2) == (side == "1")
    assert len(rg.sides) == len(rg.graphs)
    assert [u for u in rg.seg_reduce if u is not None] == rg.splits + [graphed.module.numel]
    assert len(rg.splits) == (3 if segments == "stage" else 0)
    ex = graphed.exposed_comm_ms()
    assert ex is not None and 0.0 <= ex < 1000.0, ex


def test_native_dataparallel_bottleneck_replay_records_grams_as_side_graphs(monkeypatch):
    """Bottleneck replicas (ResNet-50 at 64 px) in conv mode: the forward-time Gram work of every
    tail fold is recorded as a side graph of its own (forked inside a segment graph, the runtime
    replayed it on the main queue), and the replayed step stays bit-identical to the eager one."""
    monkeypatch.setenv("PDA_DP_SEGMENTS", "0")
    monkeypatch.setenv("PDA_DP_SIDE", "conv")
    from pytorch_distributed_amd.data import SyntheticImageNet
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    from pytorch_distributed_amd.parallel import DataParallel
    torch.manual_seed(0)
    sd = build_model("resnet50").state_dict()
    dps = []
    for _ in range(2):
        r = build_model("resnet50")
        r.load_state_dict(sd)
        dps.append(DataParallel(NativeResNet(r, device=DEV, image_size=64), device_ids=[0, 0]))
    eager, graphed = dps
    m = graphed.module
    nfold = sum(1 for b in m.blocks if len(b.units) == 3 and m._tail_fold_ok(b, 8)) \
        if m.bn_fold_wg else 0
    assert nfold > 0
    gen = eager.module.input_generator(SyntheticImageNet("train", image_size=64))
    oe = eager.make_optimizer(lr=0.05, momentum=0.9, weight_decay=1e-4)
    og = graphed.make_optimizer(lr=0.05, momentum=0.9, weight_decay=1e-4)
    for step in range(3):
        x, y = gen(torch.arange(16) + 16 * step)
        le = eager.train_step(x, y, oe, graph=False)
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            lg = graphed.train_step(x, y, og)
        assert not [w for w in caught if "Graph is empty" in str(w.message)], step
        torch.cuda.synchronize()
        assert le.item() == lg.item(), (step, le.item(), lg.item())
        assert torch.equal(eager.module.flat_grad, graphed.module.flat_grad), step
        assert torch.equal(eager.module.flat_params, graphed.module.flat_params), step
    rg = graphed._graphs[0]
    nside = sum(g is not None for g in rg.sides)
    nconv = sum(len(b.units) + (b.ds is not None and bool(m._tail_fold_ok(b, 8)))
                for b in m.blocks) + 2
    assert nside == nconv + nfold, (nside, nconv, nfold)


def test_native_dataparallel_segment_mismatch_falls_back(monkeypatch):
    """The first segmented replay verifies that every replica holds the same summed gradient; a
    mismatch (forced here: the checksum reports a different value for one replica) must not break
    the step -- it returns this step's loss, warns, re-syncs the replicas from replica 0, and the
    next step re-captures ONE graph per replica (one all-reduce after backward) and trains on."""
    monkeypatch.setenv("PDA_DP_SEGMENTS", "stage")
    monkeypatch.setenv("PDA_DP_SIDE", "0")
    from pytorch_distributed_amd import bench_step
    from pytorch_distributed_amd.data import SyntheticImageNet
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    from pytorch_distributed_amd.parallel import DataParallel
    torch.manual_seed(0)
    dp = DataParallel(NativeResNet(build_model("resnet18"), device=DEV, image_size=64),
                      device_ids=[0, 0])
    opt = dp.make_optimizer(lr=0.05, momentum=0.9, weight_decay=1e-4)
    gen = dp.module.input_generator(SyntheticImageNet("train", image_size=64))
    real = bench_step.tensor_checksum
    calls = []

    def skewed(ts):
        calls.append(1)
        c = real(ts)
        return c + 1 if len(calls) == 2 else c      # the second replica "differs"
    monkeypatch.setattr(bench_step, "tensor_checksum", skewed)
    x, y = gen(torch.arange(16))
    dp.train_step(x, y, opt)             # first step: eager + capture (the replays verify)
    x, y = gen(torch.arange(16) + 16)
    with pytest.warns(RuntimeWarning, match="falling back"):
        l1 = dp.train_step(x, y, opt)    # first segmented replay: the forced mismatch
    torch.cuda.synchronize()
    assert torch.isfinite(l1).item()
    assert dp._graphs is None and dp._force_single_segment
    assert torch.equal(dp.module.flat_params, dp.replicas[0].flat_params)
    for step in (2, 3):                  # re-capture without split points, then replay
        x, y = gen(torch.arange(16) + 16 * step)
        ls = dp.train_step(x, y, opt)
        torch.cuda.synchronize()
        assert torch.isfinite(ls).item()
        assert len(dp._graphs[0].graphs) == 1 and dp._graphs[0].splits == []
        assert torch.equal(dp.module.flat_params, dp.replicas[0].flat_params)


def test_native_dataparallel_resume_reloads_every_replica():
    """Resuming a DataParallel run (trainer.load_model_state, used by run()) must put the
    checkpoint weights into EVERY replica, not only replica 0."""
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    from pytorch_distributed_amd.parallel import DataParallel
    from pytorch_distributed_amd.trainer import load_model_state
    torch.manual_seed(0)
    dp = DataParallel(NativeResNet(build_model("resnet18"), device=DEV, image_size=64),
                      device_ids=[0, 0])
    torch.manual_seed(123)                      # a different "checkpoint"
    ck = NativeResNet(build_model("resnet18"), device=DEV, image_size=64)
    assert not torch.equal(dp.module.flat_params, ck.flat_params)
    load_model_state(dp, ck.state_dict())
    torch.cuda.synchronize()
    assert torch.equal(dp.module.flat_params, ck.flat_params)
    assert torch.equal(dp.replicas[0].flat_params, ck.flat_params)
    assert torch.equal(dp.replicas[0].flat_shadow, ck.flat_shadow)


def test_rccl_group_single_device_collectives():
    """The in-process RCCL group (ncclCommInitAll, the DataParallel gradient path over distinct
    GPUs) on the one device of the box: all_reduce (sum / avg), broadcast and reduce run through
    the native C ABI on every dtype the DP step uses, with world-1 semantics (identity), and the
    group closes cleanly. (The multi-device form runs only where several GPUs are visible.)"""
    from pytorch_distributed_amd.parallel.rccl import RcclGroup
    g = RcclGroup([0])
    try:
        for dt in (torch.float32, torch.bfloat16, torch.int64):
            t = (torch.arange(1000, device=DEV) - 300).to(dt)
            ref = t.clone()
            g.all_reduce([t], op="sum")
            g.broadcast([t], root=0)
            g.reduce([t], root=0, op="sum")
            torch.cuda.synchronize()
            assert torch.equal(t, ref), dt
        f = torch.randn(4096, device=DEV)
        ref = f.clone()
        g.all_reduce([f], op="avg")
        torch.cuda.synchronize()
        assert torch.equal(f, ref)
    finally:
        g.close()


def test_dataparallel_without_single_queue_graphs_runs_eagerly():
    """Without the single-queue graph launch (DEBUG_HIP_FORCE_GRAPH_QUEUES unset: HIP's multi-queue
    default, see runtime/graphs.py) DataParallel does not replay graphs: graph_step_ok() is False
    with a warning and train_step launches eagerly, with the same result as the graph-replay-free
    schedule. In a child process (the variable is read when HIP starts)."""
    import os
    import subprocess
    import sys
    code = r'''
import warnings, torch
from pytorch_distributed_amd.data import SyntheticImageNet
from pytorch_distributed_amd.models import build_model
from pytorch_distributed_amd.models.native import NativeResNet
from pytorch_distributed_amd.parallel import DataParallel
dev = torch.device("cuda", 0)
torch.manual_seed(0)
sd = build_model("resnet18").state_dict()
dps = []
for _ in range(2):
    r = build_model("resnet18"); r.load_state_dict(sd)
    dps.append(DataParallel(NativeResNet(r, device=dev, image_size=64), device_ids=[0, 0]))
a, b = dps
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    ok = a.graph_step_ok()
assert not ok and any("graph replay disabled" in str(x.message) for x in w), [str(x.message) for x in w]
oa, ob = a.make_optimizer(lr=0.05), b.make_optimizer(lr=0.05)
gen = a.module.input_generator(SyntheticImageNet("train", image_size=64))
for step in range(2):
    x, y = gen(torch.arange(16) + 16 * step)
    la = a.train_step(x, y, oa)            # graph=True requested, eager because of the setting
    lb = b.train_step(x, y, ob, graph=False)
    torch.cuda.synchronize()
    assert la.item() == lb.item(), (la.item(), lb.item())
    assert torch.equal(a.module.flat_params, b.module.flat_params)
assert a._graphs[0].graph is None
print("EAGER_OK")
'''
    env = dict(os.environ)
    env.pop("DEBUG_HIP_FORCE_GRAPH_QUEUES", None)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "EAGER_OK" in r.stdout, (r.stdout[-2000:] + r.stderr[-3000:])


def test_dataparallel_graph_replay_under_default_graph_queues():
    """The DataParallel replica graphs replayed under HIP's DEFAULT graph launch (the variable
    unset: a graph's independent branches go to the runtime's internal streams), with the framework's
    gate bypassed: 40 graphed steps (per-block side graphs + stage segments, two replicas on one
    device) equal to the eager schedule bit for bit. Evidence for runtime/graphs.py: the replay
    itself is correct under the default; the single-queue setting is kept for the long-session
    crash recorded in profiles/ab_r4.md section 7 (profiles/ab_r5.md section 7)."""
    import os
    import subprocess
    import sys
    code = r'''
import os, torch
assert os.environ.get("DEBUG_HIP_FORCE_GRAPH_QUEUES") is None
import pytorch_distributed_amd.runtime.graphs as G
G.single_queue_graphs = lambda: True          # bypass the gate: replay under the default
from pytorch_distributed_amd.data import SyntheticImageNet
from pytorch_distributed_amd.models import build_model
from pytorch_distributed_amd.models.native import NativeResNet
from pytorch_distributed_amd.parallel import DataParallel
dev = torch.device("cuda", 0)
torch.manual_seed(0)
sd = build_model("resnet18").state_dict()
dps = []
for _ in range(2):
    r = build_model("resnet18"); r.load_state_dict(sd)
    dps.append(DataParallel(NativeResNet(r, device=dev, image_size=64), device_ids=[0, 0]))
g, e = dps
assert g.graph_step_ok()
og, oe = g.make_optimizer(lr=0.05, momentum=0.9), e.make_optimizer(lr=0.05, momentum=0.9)
gen = g.module.input_generator(SyntheticImageNet("train", image_size=64))
for step in range(40):
    x, y = gen(torch.arange(16) + 16 * step)
    lg = g.train_step(x, y, og)
    le = e.train_step(x, y, oe, graph=False)
    torch.cuda.synchronize()
    assert lg.item() == le.item(), (step, lg.item(), le.item())
assert torch.equal(g.module.flat_params, e.module.flat_params)
assert g._graphs[0].graph is not None and len(g._graphs[0].graphs) > 1
print("DEFAULT_QUEUES_OK", len(g._graphs[0].graphs), "segment graphs per replica")
'''
    env = dict(os.environ)
    env.pop("DEBUG_HIP_FORCE_GRAPH_QUEUES", None)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "DEFAULT_QUEUES_OK" in r.stdout, (r.returncode, r.stdout[-2000:] + r.stderr[-3000:])
