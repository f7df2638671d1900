"""runtime/graphs.py: the single-queue graph launch is trusted only if DEBUG_HIP_FORCE_GRAPH_QUEUES
was "1" before the HIP runtime started (it reads the variable once). torch.cuda.device_count() /
is_available() start the runtime without torch.cuda.is_initialized() turning True, so the module
detects the runtime from the process's open /dev/kfd instead."""
from pytorch_distributed_amd.runtime import graphs


def test_value_set_after_runtime_start_is_not_trusted(monkeypatch):
    monkeypatch.delenv(graphs.GRAPH_QUEUES_VAR, raising=False)
    started = [False]
    monkeypatch.setattr(graphs, "hip_runtime_started", lambda: started[0])
    assert graphs.single_queue_graphs() is False          # observed unset before the start
    started[0] = True                                      # e.g. torch.cuda.device_count()
    assert graphs.request_single_queue_graphs() is False   # too late: nothing set, not trusted
    monkeypatch.setenv(graphs.GRAPH_QUEUES_VAR, "1")       # set by hand after the start
    assert graphs.single_queue_graphs() is False


def test_value_set_before_runtime_start_is_trusted(monkeypatch):
    monkeypatch.delenv(graphs.GRAPH_QUEUES_VAR, raising=False)
    started = [False]
    monkeypatch.setattr(graphs, "hip_runtime_started", lambda: started[0])
    assert graphs.request_single_queue_graphs() is True
    started[0] = True
    assert graphs.single_queue_graphs() is True


def test_runtime_not_started_in_this_cpu_process():
    assert graphs.hip_runtime_started() is False
