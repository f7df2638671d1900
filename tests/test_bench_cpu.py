"""The driver's ``bench.py`` contract rehearsed on the CPU (gloo, no GPU): one JSON line from rank
0 with the headline keys, MAX-over-ranks timing, the N>1 self-validation keys (bucket plan,
cross-rank bit-exact weight checksum) -- and a rank whose weights diverge makes the run exit
non-zero (``PDA_BENCH_PERTURB_RANK`` test hook)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--device", "cpu", "--arch", "resnet18", "--batch", "2", "--image-size", "32",
        "--steps", "2", "--warmup", "1", "--dtype", "fp32", "--fp32-steps", "0", "--dp-steps", "0"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(nproc, extra_env=None, tmp=None, extra_args=()):
    env = dict(os.environ)
    env.update({"OMP_NUM_THREADS": "2", "PDA_BIND_NUMA": "0"})
    env.update(extra_env or {})
    if nproc == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), *ARGS, *extra_args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
               str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(_port()),
               os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), *ARGS, *extra_args]
    return subprocess.run(cmd, cwd=tmp, env=env, capture_output=True, text=True, timeout=600)


def _record(r):
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr[-3000:]
    return json.loads(lines[0])


def test_bench_cpu_single(tmp_path):
    r = _run(1, tmp=tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == 1 and rec["steps"] == 2 and rec["warmup"] == 1
    assert abs(rec["value"] - 2 * 1000.0 / rec["ms_per_step"]) / rec["value"] < 1e-2


def test_bench_cpu_two_ranks_self_validation(tmp_path):
    r = _run(2, tmp=tmp_path)
    assert r.returncode == 0, r.stderr[-4000:]
    rec = _record(r)
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 4
    assert rec["config"]["parallelism"] == "dp2"
    assert rec["weights_consistent"] is True
    assert rec["buckets"] >= 1 and len(rec["bucket_bytes"]) == rec["buckets"]
    assert sum(rec["bucket_bytes"]) >= 11_000_000 * 4     # every ResNet-18 gradient is bucketed
    assert rec["comm"] == "ProcessGroupCommunicator"
    # measured all-reduce cost of the gradient communicator (the reducer's alpha / bandwidth)
    pr = rec["xgmi_probe"]
    assert pr["comm"] == "ProcessGroupCommunicator" and len(pr["ms"]) == len(pr["bytes"])
    assert all(v > 0 for v in pr["ms"]) and pr["alpha_us"] > 0 and pr["busbw_GBs"] > 0
    # the resnet_ddp_apex.py configuration, timed after the headline on every rank
    assert rec["amp_fp16_images_per_sec"] > 0 and rec["amp_weights_consistent"] is True
    assert "DDP" in rec["amp_config"]
    assert isinstance(rec["comm_env"], dict) and rec["numa_bound"] is False
    assert "gpu_util_pct" in rec
    # per-rank timed-region spread of each timed pass (a straggler rank is visible)
    sp = rec["rank_time_spread"]
    for k in ("headline", "amp_fp16"):
        assert 0 < sp[k]["min_s"] <= sp[k]["max_s"] and sp[k]["spread_pct"] >= 0
    assert abs(sp["headline"]["max_s"] * 1000.0 / rec["steps"] - rec["ms_per_step"]) < 0.1
    assert rec["amp_dtype"] == "fp16"


def test_bench_cpu_four_ranks(tmp_path):
    """World 4 (the driver's 8-GPU run has more ranks than any other rehearsal): one record, every
    rank in the timing spread, weights bit-identical on all four ranks."""
    r = _run(4, tmp=tmp_path, extra_args=("--amp-steps", "0", "--comm-probe", "0"))
    assert r.returncode == 0, r.stderr[-4000:]
    rec = _record(r)
    assert rec["n_gpus"] == 4 and rec["config"]["global_batch"] == 8
    assert rec["config"]["parallelism"] == "dp4"
    assert rec["weights_consistent"] is True
    assert abs(rec["value"] - 8 * 1000.0 / rec["ms_per_step"]) / rec["value"] < 1e-2
    sp = rec["rank_time_spread"]["headline"]
    assert 0 < sp["min_s"] <= sp["max_s"]


def test_bench_cpu_eight_ranks(tmp_path):
    """World 8 -- the rank count of the driver's one-node scaling run: one record, all eight ranks
    in the timing spread, weights bit-identical on every rank, and the DataParallel pass's hand-off
    (rank 0 runs ``bench.py --dp`` as a child process while ranks 1-7 wait on the TCP store for its
    keys) rehearsed on the CPU."""
    r = _run(8, tmp=tmp_path, extra_args=("--amp-steps", "0", "--comm-probe", "0", "--dp-steps", "2"))
    assert r.returncode == 0, r.stderr[-4000:]
    rec = _record(r)
    assert rec["n_gpus"] == 8 and rec["config"]["global_batch"] == 16
    assert rec["config"]["parallelism"] == "dp8"
    assert rec["weights_consistent"] is True
    assert abs(rec["value"] - 16 * 1000.0 / rec["ms_per_step"]) / rec["value"] < 1e-2
    sp = rec["rank_time_spread"]["headline"]
    assert 0 < sp["min_s"] <= sp["max_s"] and sp["spread_pct"] >= 0
    assert "dp_error" not in rec, rec.get("dp_error")
    assert rec["dp_images_per_sec"] > 0 and rec["dp_replicas_consistent"] is True
    assert rec["dp_config"].startswith("dataparallel1")


def test_bench_cpu_eight_ranks_diverged_rank_fails(tmp_path):
    """At world 8 a single rank whose weights diverge (rank 5) still fails the run."""
    r = _run(8, {"PDA_BENCH_PERTURB_RANK": "5"}, tmp=tmp_path,
             extra_args=("--amp-steps", "0", "--comm-probe", "0"))
    assert r.returncode != 0
    assert "parameters differ across ranks" in r.stderr


def test_numa_binding_precedes_any_hip_call(monkeypatch, tmp_path):
    """bench.py binds a rank to its GPU's NUMA node before HIP starts (its runtime threads inherit
    the affinity the process has then): the GPU count comes from the KFD topology in sysfs, and no
    torch.cuda entry point that initialises HIP runs before bind_numa."""
    import importlib.util
    import torch
    from pytorch_distributed_amd import launch
    # a fake KFD topology: one CPU node, two GPU nodes
    for i, simd in enumerate((0, 304, 304)):
        d = tmp_path / "nodes" / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"simd_count {simd}\ndomain 0\nlocation_id {256 * (i + 1)}\n")
    monkeypatch.setattr(launch, "_KFD_ROOT", str(tmp_path / "nodes"))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    calls = []

    def no_hip(name):
        def f(*a, **k):
            raise AssertionError(f"torch.cuda.{name} called before the NUMA binding")
        return f
    for name in ("device_count", "is_available", "init", "_lazy_init", "set_device",
                 "current_device", "synchronize"):
        monkeypatch.setattr(torch.cuda, name, no_hip(name))
    monkeypatch.setattr(launch, "bind_numa", lambda lr: calls.append(lr) or True)
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.delenv("PDA_BIND_NUMA", raising=False)
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    args = type("A", (), {"nccl_channels": 0, "nccl_proto": "", "nccl_algo": "", "device": "cuda"})()
    out = bench._configure_process(args)
    assert calls == [1] and out["numa_bound"] is True
    assert launch.visible_gpu_count() == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert launch.visible_gpu_count() == 1
    assert launch.gpu_pci_bdf(0) == "0000:03:00.0"     # visible 0 = physical GPU 1 (node 2)


def test_visible_gpu_count_render_nodes_and_selectors(monkeypatch, tmp_path):
    """The launcher's GPU count (no HIP call): a KFD node counts only when its render node is
    accessible (sysfs lists every GPU of the host inside a container given only some); HIP applies
    HIP_VISIBLE_DEVICES, or CUDA_VISIBLE_DEVICES only without it; a UUID selector is counted by torch
    in a child process, never taken as 'no filter'."""
    from pytorch_distributed_amd import launch
    dri = tmp_path / "dri"
    dri.mkdir()
    for i, simd in enumerate((0, 304, 304, 304, 304)):
        d = tmp_path / "nodes" / str(i)
        d.mkdir(parents=True)
        minor = 127 + i if simd else 0
        (d / "properties").write_text(f"simd_count {simd}\ndomain 0\nlocation_id {256 * (i + 1)}\n"
                                      f"drm_render_minor {minor}\n")
    for minor in (128, 130):          # the container may open GPU nodes 1 and 3 only
        (dri / f"renderD{minor}").write_text("")
    monkeypatch.setattr(launch, "_KFD_ROOT", str(tmp_path / "nodes"))
    monkeypatch.setattr(launch, "_DRI_ROOT", str(dri))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert launch.visible_gpu_count() == 2
    assert launch.gpu_pci_bdf(1) == "0000:04:00.0"    # the second accessible GPU = KFD node 3
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "1")
    assert launch.visible_gpu_count() == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")  # HIP reads this one, not CUDA_VISIBLE_DEVICES
    assert launch.visible_gpu_count() == 2
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1")   # applied first: one device left, index 0
    assert launch.visible_gpu_count() == 1
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "GPU-0123456789abcdef")
    monkeypatch.setattr(launch, "_child_device_count", lambda: 7)
    assert launch.visible_gpu_count() == 7
    assert launch.gpu_pci_bdf(0) is None


def _run_bare(gpus, extra_args=(), extra_env=None, tmp=None, device_args=ARGS):
    """bench.py started the way the driver starts ``--gpus 1``: no external launcher."""
    env = dict(os.environ)
    env.update({"OMP_NUM_THREADS": "1", "PDA_BIND_NUMA": "0"})
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(extra_env or {})
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), *device_args,
           *extra_args]
    return subprocess.run(cmd, cwd=tmp, env=env, capture_output=True, text=True, timeout=600)


def test_bench_bare_gpus8_self_launches_ranks(tmp_path):
    """``python bench.py --gpus 8`` with NO external launcher still runs 8 ranks (the parent starts
    torch.distributed.run as a child before any HIP call) and relays ONE record from rank 0."""
    r = _run_bare(8, ("--amp-steps", "0", "--comm-probe", "0"), tmp=tmp_path)
    assert r.returncode == 0, r.stderr[-4000:]
    rec = _record(r)
    assert rec["n_gpus"] == 8 and rec["config"]["parallelism"] == "dp8"
    assert rec["config"]["global_batch"] == 16
    assert rec["weights_consistent"] is True
    assert rec["launcher"].startswith("bench.py -> torch.distributed.run")
    sp = rec["rank_time_spread"]["headline"]
    assert 0 < sp["min_s"] <= sp["max_s"]


def test_bench_bare_diverged_rank_exit_code_relayed(tmp_path):
    """A failing rank under the self-launch makes the parent exit non-zero."""
    r = _run_bare(2, ("--amp-steps", "0", "--comm-probe", "0"), {"PDA_BENCH_PERTURB_RANK": "1"},
                  tmp=tmp_path)
    assert r.returncode != 0
    assert "parameters differ across ranks" in r.stderr


def test_bench_refuses_more_gpus_than_visible(tmp_path):
    """``--gpus 2`` where fewer GPUs are visible (none in this container) exits non-zero at once with
    the device-count message instead of folding ranks onto one device."""
    import time
    t0 = time.time()
    r = _run_bare(2, tmp=tmp_path, device_args=("--steps", "1", "--warmup", "0"),
                  extra_env={"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": ""})
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs 2 visible GPUs" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert time.time() - t0 < 120


def test_bench_refuses_world_size_mismatch(tmp_path):
    """Started by a launcher whose world differs from --gpus: refused, not mislabelled."""
    r = _run_bare(4, tmp=tmp_path, extra_env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE 2 but --gpus 4" in r.stderr


def test_bench_cpu_diverged_rank_fails(tmp_path):
    r = _run(2, {"PDA_BENCH_PERTURB_RANK": "1"}, tmp=tmp_path)
    assert r.returncode != 0
    assert "parameters differ across ranks" in r.stderr
