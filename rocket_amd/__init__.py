"""rocket_amd — an MI355X-native training-loop engine with the capability set of dsenushkin/rocket.

A pipeline is a tree of capsules (``Launcher → Looper → {Dataset, Module →
{Loss, Optimizer, Scheduler, Meter → Metric}, Checkpointer, Tracker}``) that
exchange data through one :class:`Attributes` buffer and react to the
``setup/set/launch/reset/destroy`` events.  Underneath, the runtime is native to
AMD Instinct MI355X (gfx950): PyTorch-ROCm for autograd, hand-written CDNA4 HIP
kernels for the hot ops (:mod:`rocket_amd.ops`), RCCL over xGMI for data
parallelism (:mod:`rocket_amd.parallel`) and HIP graphs for launch-bound steps.
"""

from rocket_amd.runtime import hipenv as _hipenv  # noqa: F401  (before any HIP initialisation)
from rocket_amd.core import (  # noqa: F401
    Attributes,
    Capsule,
    Checkpointer,
    Dataset,
    Dispatcher,
    Events,
    Launcher,
    Looper,
    Loss,
    Meter,
    Metric,
    Module,
    Optimizer,
    Scheduler,
    Tracker,
)
from rocket_amd.runtime.data import DeviceTensorDataset  # noqa: F401
from rocket_amd.runtime.host_data import HostTensorDataset  # noqa: F401
from rocket_amd.runtime.engine import Engine  # noqa: F401

__version__ = "0.1.0"

__all__ = [
    "Attributes",
    "Events",
    "Capsule",
    "Dispatcher",
    "Launcher",
    "Looper",
    "Dataset",
    "Module",
    "Loss",
    "Optimizer",
    "Scheduler",
    "Checkpointer",
    "Tracker",
    "Meter",
    "Metric",
    "Engine",
    "DeviceTensorDataset",
]
