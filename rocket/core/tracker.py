"""Reference ``rocket/core/tracker.py``: Tracker."""

from rocket_amd.core.tracker import Tracker  # noqa: F401
