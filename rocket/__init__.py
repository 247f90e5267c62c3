"""Import-path compatibility for code written against the reference (``import rocket``).

The reference exposes its capsules as ``rocket.<Class>`` and its modules as
``rocket.core.<module>`` / ``rocket.utils.<module>`` (``rocket/__init__.py:1``,
``rocket/core/__init__.py:1-12``).  This package keeps those names and points them at the
MI355X-native implementation in :mod:`rocket_amd`, so a reference training script runs unchanged.
"""

from rocket.core import *  # noqa: F401,F403
from rocket_amd import DeviceTensorDataset, Engine, HostTensorDataset  # noqa: F401
from rocket_amd import __version__  # noqa: F401
