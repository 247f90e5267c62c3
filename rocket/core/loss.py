"""Reference ``rocket/core/loss.py``: Loss."""

from rocket_amd.core.objectives import Loss  # noqa: F401
