"""Capsule layer (reference ``rocket/core``)."""

from rocket_amd.core.attributes import Attributes
from rocket_amd.core.capsule import Capsule, Events
from rocket_amd.core.checkpointer import Checkpointer
from rocket_amd.core.dataset import Dataset
from rocket_amd.core.dispatcher import Dispatcher
from rocket_amd.core.launcher import Launcher
from rocket_amd.core.looper import Looper
from rocket_amd.core.meter import Meter, Metric
from rocket_amd.core.module import Module
from rocket_amd.core.objectives import Loss, Optimizer, Scheduler
from rocket_amd.core.tracker import Tracker

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
]
