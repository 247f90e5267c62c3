"""Reference ``rocket/core/meter.py``: Meter, Metric, rebuild_batch."""

from rocket_amd.core.meter import Meter, Metric, rebuild_batch  # noqa: F401
