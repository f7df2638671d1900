"""``hfai.client`` equivalent: the preemption ("suspend") protocol (reference ``restnet_ddp.py:35-47``).

``receive_suspend_command()`` is True once the scheduler asked this process to stop (SIGUSR1,
the ``MX_SUSPEND_FILE`` sentinel, or ``MX_SUSPEND_AT_STEP`` for tests); ``go_suspend()`` exits with
the requeue code so the job is restarted and resumes from ``latest.pt``.
"""
from ..utils.suspend import REQUEUE_EXIT_CODE, go_suspend, receive_suspend_command

__all__ = ["receive_suspend_command", "go_suspend", "REQUEUE_EXIT_CODE"]
