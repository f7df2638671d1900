"""``hfai.nccl`` equivalent."""
from . import distributed  # noqa: F401
