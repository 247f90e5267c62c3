"""Reference ``rocket/core/loop.py``: Looper."""

from rocket_amd.core.looper import Looper  # noqa: F401
