"""``hfai.nn`` equivalent."""
from . import parallel  # noqa: F401
