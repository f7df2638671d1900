from .checkpoint import load_latest, save_best, save_latest
from .metrics import MetricsLog, Throughput
from .suspend import REQUEUE_EXIT_CODE, SuspendMonitor, go_suspend, receive_suspend_command

__all__ = ["load_latest", "save_best", "save_latest", "MetricsLog", "Throughput",
           "REQUEUE_EXIT_CODE", "SuspendMonitor", "go_suspend", "receive_suspend_command"]
