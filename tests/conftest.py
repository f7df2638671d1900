import os
import sys

import pytest

# the GPU session replays HIP graphs (DataParallel replicas, whole-step graphs): single-queue graph
# launch, set before HIP starts (pytorch_distributed_amd/runtime/graphs.py GRAPH_QUEUES_VAR)
os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import pytorch_distributed_amd  # noqa: E402,F401


def pytest_configure(config):
    if os.environ.get("PDA_SEGV_BT"):   # diagnostic: native backtrace on a segfault
        import ctypes
        ctypes.CDLL(os.environ["PDA_SEGV_BT"]).segv_bt_install()
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _gpu_test_isolation(request):
    """After each GPU test: drop its objects (HIP graphs, streams' tensors, workspaces) and return
    the caching allocator's blocks, so one long session's earlier tests leave no state behind.
    PDA_TEST_MEMLOG=1 prints the device's free memory before each GPU test."""
    gpu = "gpu" in request.keywords
    if gpu and os.environ.get("PDA_TEST_MEMLOG") == "1":
        import torch
        free, total = torch.cuda.mem_get_info()
        print(f"\n[mem] {request.node.nodeid}: free {free / 2**30:.1f} / {total / 2**30:.1f} GiB, "
              f"reserved {torch.cuda.memory_reserved() / 2**30:.1f} GiB", flush=True)
    yield
    if gpu:
        import gc
        import torch
        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
