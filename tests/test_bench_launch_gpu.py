"""The driver's multi-GPU bench contract, rehearsed on one GPU: ``bench.py`` launched by
``torch.distributed.run`` with 2 ranks (gloo stands in for RCCL, which refuses two ranks on one
device). Covers env-rank parsing, the DDP-wrapped native step, the barrier/synchronize timing
bracket, the MAX-over-ranks elapsed time and the single JSON line from rank 0."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_torchrun_two_ranks(tmp_path):
    env = dict(os.environ)
    env.update({"PDA_DIST_BACKEND": "gloo", "PDA_BIND_NUMA": "0", "OMP_NUM_THREADS": "4",
                "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse-fold", "--steps", "2", "--warmup", "1",
           "--batch", "16", "--image-size", "64"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["config"]["global_batch"] == 32 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["engine"] == "native" and rec["config"]["hip_graph"] is False
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    assert abs(rec["value"] - 32 * 1000.0 / rec["ms_per_step"]) / rec["value"] < 1e-2
    assert rec["loss"] == rec["loss"]         # finite, not NaN
    # N>1 self-validation (driver's first multi-GPU run must prove itself)
    assert rec["weights_consistent"] is True
    assert rec["buckets"] >= 3 and len(rec["bucket_bytes"]) == rec["buckets"]
    assert all(b % (8 * 7 * 256) == 0 for b in rec["bucket_bytes"])
    assert rec["comm"] == "ProcessGroupCommunicator" and rec["rccl_world"] is None   # gloo here
    pr = rec["xgmi_probe"]                    # device tensors through the gradient communicator
    assert len(pr["ms"]) == len(pr["bytes"]) and all(v > 0 for v in pr["ms"])
    # the default fp32 pass (split convs, >= TF32 precision) and the exact-f32 MFMA pass
    assert rec["fp32_images_per_sec"] > 0 and rec["fp32_engine"] == "native"
    assert rec["fp32_conv"].startswith("split") and rec["fp32_exact_images_per_sec"] > 0
    # the other GPU configurations of BASELINE.json, each labelled with its config/dtype:
    # fp16 AMP-DDP (resnet_ddp_apex.py) on both ranks, DataParallel (resnet_dp.py) by rank 0
    # over the visible devices (one here) while rank 1 waits on the store
    assert rec["amp_fp16_images_per_sec"] > 0 and rec["amp_weights_consistent"] is True
    assert "fp16" in rec["amp_config"] and "DDP" in rec["amp_config"]
    assert rec["dp_images_per_sec"] > 0 and rec["dp_replicas_consistent"] is True
    assert rec["dp_config"].startswith("dataparallel1")
    assert "HSA_ENABLE_IPC_MODE_LEGACY" in rec["comm_env"]
    assert rec["max_mem_gb"] > 0 and rec["amp_max_mem_gb"] > 0 and rec["dp_max_mem_gb"] > 0


def test_bench_torchrun_perturbed_rank_fails(tmp_path):
    env = dict(os.environ)
    env.update({"PDA_DIST_BACKEND": "gloo", "PDA_BIND_NUMA": "0", "OMP_NUM_THREADS": "4",
                "HSA_ENABLE_IPC_MODE_LEGACY": "0", "PDA_BENCH_PERTURB_RANK": "1"})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse-fold", "--steps", "1", "--warmup", "1",
           "--batch", "8", "--image-size", "64", "--fp32-steps", "0", "--amp-steps", "0",
           "--dp-steps", "0"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "parameters differ across ranks" in r.stderr


def test_bench_bare_gpus2_refused_on_one_gpu_box(tmp_path):
    """The driver's invocation form, ``python bench.py --gpus 2`` with no launcher, on a box with one
    visible GPU: a non-zero exit with the device-count message within seconds (no HIP call made),
    never a silent one-GPU record."""
    import time
    from pytorch_distributed_amd.launch import visible_gpu_count
    if visible_gpu_count() >= 2:
        pytest.skip("more than one GPU visible")
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0"], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs 2 visible GPUs" in r.stderr and time.time() - t0 < 60
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
