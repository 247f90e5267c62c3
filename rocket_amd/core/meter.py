"""Evaluation metering: cross-rank gather of selected batch entries, then user metrics.

Parity (reference ``rocket/core/meter.py``):

* ``Meter(capsules, keys, priority=1000)`` sorts ``keys`` (``:54-61``);
* ``launch`` runs only with grad disabled, gathers ``attrs.batch[key]`` for every
  key with ``gather_for_metrics`` (all-gather + truncation of the wrap-around
  padding on the last batch), rebuilds the batch with the gathered entries and
  launches the child metrics on every rank (``:63-105``);
* ``Metric(priority)`` records ``_step = epoch_idx`` in ``set``; ``launch`` and
  ``reset`` are abstract (``:108-206``).
"""

from __future__ import annotations

from typing import List

import torch

from rocket_amd.core.attributes import Attributes
from rocket_amd.core.capsule import Capsule
from rocket_amd.core.dispatcher import Dispatcher
from rocket_amd.utils.collections import apply_to_collection


def rebuild_batch(lookup_table: dict):
    def fn(value, key, **kwargs):
        return lookup_table.get(key, value)

    return fn


class Meter(Dispatcher):
    def __init__(self, capsules: List[Capsule], keys: List, priority: int = 1000) -> None:
        super().__init__(capsules=capsules, priority=priority)
        self._keys = sorted(keys)

    def launch(self, attrs: Attributes | None = None) -> None:
        if attrs is None or attrs.batch is None:
            return
        if torch.is_grad_enabled():
            return
        values = [attrs.batch[k] for k in self._keys]
        gathered = self._accelerator.gather_for_metrics(values)
        table = dict(zip(self._keys, gathered))
        attrs.batch = apply_to_collection(attrs.batch, rebuild_batch(table))
        Dispatcher.launch(self, attrs=attrs)


class Metric(Capsule):
    def __init__(self, priority: int = 1000) -> None:
        super().__init__(priority=priority)
        self._step = 0

    def set(self, attrs: Attributes | None = None) -> None:
        Capsule.set(self, attrs)
        self._step = attrs.launcher.epoch_idx if attrs is not None and attrs.launcher is not None else 0

    def launch(self, attrs: Attributes | None = None) -> None:
        raise NotImplementedError(f"{self.__class__.__name__}: metric should implement launch()")

    def reset(self, attrs: Attributes | None = None) -> None:
        raise NotImplementedError(f"{self.__class__.__name__}: metric should implement reset()")
