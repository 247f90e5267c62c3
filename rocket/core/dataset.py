"""Reference ``rocket/core/dataset.py``: Dataset."""

from rocket_amd.core.dataset import Dataset  # noqa: F401
