"""``rocket.core`` (reference ``rocket/core/__init__.py:1-27``) backed by :mod:`rocket_amd.core`."""

from rocket.core.capsule import Attributes, Capsule, Events  # noqa: F401
from rocket.core.checkpoint import Checkpointer  # noqa: F401
from rocket.core.dataset import Dataset  # noqa: F401
from rocket.core.dispatcher import Dispatcher  # noqa: F401
from rocket.core.launcher import Launcher  # noqa: F401
from rocket.core.loop import Looper  # noqa: F401
from rocket.core.loss import Loss  # noqa: F401
from rocket.core.meter import Meter, Metric  # noqa: F401
from rocket.core.module import Module  # noqa: F401
from rocket.core.optimizer import Optimizer  # noqa: F401
from rocket.core.scheduler import Scheduler  # noqa: F401
from rocket.core.tracker import Tracker  # noqa: F401

__sphinx_classes__ = [Capsule, Dispatcher, Dataset, Module, Loss, Optimizer, Scheduler, Tracker, Checkpointer,
                      Meter, Metric]
