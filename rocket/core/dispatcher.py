"""Reference ``rocket/core/dispatcher.py``: Dispatcher."""

from rocket_amd.core.dispatcher import Dispatcher  # noqa: F401
