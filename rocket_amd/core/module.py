"""Model capsule: device placement, data-parallel replica, forward under AMP + GA.

Parity (reference ``rocket/core/module.py``):

* ``Module(module, capsules=[], priority=1000)`` — children are losses,
  optimizers, schedulers, post-processors (``:50-60``);
* ``setup`` dedupes against the engine's model registry, moves the model and
  prepares it (replica wrapper when W>1), then sets up children (``:62-108``);
* ``launch``: train/eval mode from ``torch.is_grad_enabled()``; inside
  ``runner()`` (autocast ⊕ accumulate) ``attrs.batch = module(attrs.batch)``
  and the children launch (``:110-142, :175-219``);
* ``destroy`` unregisters the model (``:144-171``).

Differences: a module shared by several ``Module`` capsules (train + eval
loopers) resolves to the *same* replica wrapper (Q8); forward goes through
``__call__`` so module hooks run.

Graph capture (MI355X-first, opt-in ``capture=True``): after ``warmup`` eager
iterations the whole training micro-step — forward, loss, backward, gradient
all-reduce and fused optimizer update — is captured into a HIP graph per
(sync / no-sync) variant and replayed; host-side bookkeeping of the children
(loss/lr posting, scheduler) still runs every iteration.  See
:mod:`rocket_amd.runtime.graphs`.
"""

from __future__ import annotations

import contextlib

import torch

from rocket_amd.core.attributes import Attributes
from rocket_amd.core.capsule import Capsule
from rocket_amd.core.dispatcher import Dispatcher
from rocket_amd.runtime.data import materialize_batch


class Module(Dispatcher):
    def __init__(
        self,
        module: torch.nn.Module,
        capsules: list[Capsule] | None = None,
        priority: int = 1000,
        capture: bool = False,
        warmup: int = 3,
    ) -> None:
        super().__init__(capsules=list(capsules or []), priority=priority)
        self._module = module
        self._capture = capture
        self._warmup = warmup
        self._graphs = None
        self._gathers_rows = False  # the model gathers deferred loader batches itself (PendingRows)

    @property
    def module(self) -> torch.nn.Module:
        return self._module

    def setup(self, attrs: Attributes | None = None) -> None:
        self.check_accelerator()
        engine = self._accelerator
        base = getattr(self._module, "module", self._module)
        matches = [m for m in engine._models if m is self._module or m is base]
        if len(matches) > 1:
            raise RuntimeError(f"{self.__class__.__name__}: same module has been registered twice.")
        if matches:
            self._module = engine.replica(matches[0])
        else:
            self._module = engine.prepare_model(self._module, device_placement=engine.device_placement)
        Dispatcher.setup(self, attrs)
        self._gathers_rows = bool(getattr(engine.unwrap_model(self._module), "consumes_pending_rows", False))
        if self._capture and engine.device.type == "cuda":
            from rocket_amd.runtime.graphs import StepGraphs

            self._graphs = StepGraphs(self, warmup=self._warmup)

    def launch(self, attrs: Attributes | None = None) -> None:
        if attrs is None or attrs.get("batch") is None:
            return
        if not self._gathers_rows:  # a deferred device-loader batch the model does not gather itself
            materialize_batch(attrs["batch"])
        train = torch.is_grad_enabled()
        if self._module.training != train:  # a recursive .train() costs ~20 us per iteration
            self._module.train(train)
        if self._graphs is not None and torch.is_grad_enabled() and self._graphs.launch(attrs):
            return
        with self.runner():
            attrs.batch = self._module(attrs.batch)
            Dispatcher.launch(self, attrs=attrs)

    def destroy(self, attrs: Attributes | None = None) -> None:
        engine = self._accelerator
        base = engine.unwrap_model(self._module)
        for i, m in enumerate(engine._models):
            if m is base:
                engine._models.pop(i)
                break
        if self._graphs is not None:
            self._graphs.release()  # drop graphs + memory pool, keep counters for inspection
        Dispatcher.destroy(self, attrs=attrs)

    @contextlib.contextmanager
    def runner(self):
        with self._accelerator.autocast(), self._accelerator.accumulate(self._module):
            yield
