"""Dataset capsule: owns a sharded loader and fills ``attrs.batch``.

Parity (reference ``rocket/core/dataset.py``):

* ``Dataset(dataset, statefull=True, priority=1000, **dataloader_kwargs)`` with
  ``torch_collate`` as default ``collate_fn`` (``:100-126``);
* ``setup`` dedupes by dataset identity against the engine's loaders and raises
  on a duplicate registration (``:128-180``);
* ``set`` resumes with ``skip_first_batches`` when a checkpoint restored
  ``batch_idx > 0`` and grad is enabled (``:182-213``);
* ``launch`` is a no-op when ``attrs`` is ``None`` or a batch is already present,
  sets ``looper.terminate`` on exhaustion, moves the batch to the device and
  counts ``batch_idx`` (``:240-288``); ``reset`` rewinds (``:215-238``);
* state ``{batch_idx}`` (``:328-361``).

Differences: the loader is epoch-seeded (exactly-once mid-epoch resume, Q5);
host batches are pinned and transferred one step ahead; a
:class:`~rocket_amd.runtime.data.DeviceTensorDataset` is batched on-device;
``destroy`` really unregisters the loader (Q2).
"""

from __future__ import annotations

from typing import Iterable

import torch

from rocket_amd.core.attributes import Attributes
from rocket_amd.core.capsule import Capsule
from rocket_amd.utils.torch import torch_collate, torch_move


class Dataset(Capsule):
    def __init__(self, dataset: Iterable, statefull: bool = True, priority: int = 1000, **kwargs) -> None:
        super().__init__(statefull=statefull, priority=priority)
        self._dataset = dataset
        self._dataloader = None
        self._active_dataloader = None
        self._iterator = None
        self._kwargs = kwargs
        self._kwargs.setdefault("collate_fn", torch_collate)
        self._batch_idx = 0
        self._total = 0
        self._resumed_exhausted = False

    def setup(self, attrs: Attributes | None = None) -> None:
        Capsule.setup(self, attrs=attrs)
        found = [dl for dl in self._accelerator._dataloaders if dl.dataset is self._dataset]
        if len(found) > 1:
            raise RuntimeError(f"{self.__class__.__name__}: same dataset has been registered twice.")
        if found:
            self._dataloader = found[0]
        else:
            self._dataloader = self._accelerator.make_loader(self._dataset, device_placement=True, **self._kwargs)

    def set(self, attrs: Attributes | None = None) -> None:
        Capsule.set(self, attrs=attrs)
        epoch = attrs.launcher.epoch_idx if attrs is not None and attrs.launcher is not None else None
        if epoch is not None:
            self._dataloader.set_epoch(epoch)
        self._resumed_exhausted = False
        if torch.is_grad_enabled() and self._batch_idx > 0:
            self._active_dataloader = self._accelerator.skip_first_batches(self._dataloader, self._batch_idx)
            self._resumed_exhausted = len(self._active_dataloader) == 0
        else:
            self._active_dataloader = self._dataloader
        self._total = len(self._active_dataloader)
        self._iterator = iter(self._active_dataloader)

    def reset(self, attrs: Attributes | None = None) -> None:
        Capsule.reset(self, attrs=attrs)
        self._batch_idx = 0
        self._total = 0
        self._iterator = None
        self._active_dataloader = None

    def launch(self, attrs: Attributes | None = None) -> None:
        Capsule.launch(self, attrs=attrs)
        # (per-iteration path: the buffer's keys through dict methods, not the attribute hook)
        if attrs is None or attrs.get("batch") is not None:
            return
        data = next(self._iterator, None) if self._iterator is not None else None
        looper = attrs.get("looper")
        if data is None:
            attrs["batch"] = None
            if looper is not None:
                looper["terminate"] = True
            return
        if getattr(self._active_dataloader, "device_resident", False):
            attrs["batch"] = data  # device/host loaders already delivered the batch on the device
        else:
            attrs["batch"] = torch_move(data, self._accelerator.device)
        if looper is not None:
            looper["terminate"] = False
        self._batch_idx += 1

    def destroy(self, attrs: Attributes | None = None) -> None:
        Capsule.destroy(self, attrs=attrs)
        registry = self._accelerator._dataloaders
        for i, dl in enumerate(registry):
            if dl is self._dataloader:
                registry.pop(i)
                break
        self._dataloader = None
        self._active_dataloader = None
        self._iterator = None

    def state_dict(self) -> dict:
        return dict(batch_idx=self._batch_idx)

    def load_state_dict(self, state: dict) -> None:
        self._batch_idx = state["batch_idx"]
