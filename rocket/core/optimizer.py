"""Reference ``rocket/core/optimizer.py``: Optimizer."""

from rocket_amd.core.objectives import Optimizer  # noqa: F401
