"""Reference ``rocket/core/capsule.py``: Attributes, Events, Capsule."""

from rocket_amd.core.attributes import Attributes  # noqa: F401
from rocket_amd.core.capsule import Capsule, Events  # noqa: F401
