"""Reference ``rocket/core/scheduler.py``: Scheduler."""

from rocket_amd.core.objectives import Scheduler  # noqa: F401
