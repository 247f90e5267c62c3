"""Reference ``rocket/core/checkpoint.py``: Checkpointer."""

from rocket_amd.core.checkpointer import Checkpointer  # noqa: F401
