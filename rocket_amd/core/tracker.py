"""Tracker capsule: drains ``attrs.tracker`` into an experiment-tracking backend.

Parity (reference ``rocket/core/tracker.py``):

* ``Tracker(backend='tensorboard', config=None, priority=200)`` — priority 200
  runs it after Dataset/Module (1000) and before the Checkpointer (100);
* ``setup`` resolves the backend (an instance is used as-is; a name is looked up
  and initialised on demand) (``:64-105``);
* ``set`` creates ``attrs.tracker = {scalars: [], images: []}``; producers append
  ``Attributes(step, data)`` records (``loss.py:103-109``, ``optimizer.py:134-142``);
* records are logged on rank 0 only, images then scalars (``:201-254``).

Difference: the reference flushes every iteration, which — with device-side
values — would synchronise host and GPU once per step.  Records are buffered and
flushed every ``flush_every`` iterations (and always at ``reset``); all pending
device values of a flush come back in one copy.  Logged steps and values are
identical, only written later.  ``reset`` always clears the buffer (Q11).
"""

from __future__ import annotations

from typing import List

from rocket_amd.core.attributes import Attributes
from rocket_amd.core.capsule import Capsule
from rocket_amd.runtime.trackers import GeneralTracker
from rocket_amd.utils.lazy import materialize, plain


class Tracker(Capsule):
    def __init__(self, backend="tensorboard", config: dict | None = None, priority: int = 200,
                 flush_every: int = 50) -> None:
        super().__init__(priority=priority)
        self._backend = backend
        self._tracker = None
        self._config = config or None
        self._flush_every = max(1, int(flush_every))
        self._pending_images: List[Attributes] = []
        self._pending_scalars: List[Attributes] = []
        self._iters = 0

    def setup(self, attrs: Attributes | None = None) -> None:
        Capsule.setup(self, attrs=attrs)
        engine = self._accelerator
        if not isinstance(self._backend, str) and hasattr(self._backend, "log"):
            self._tracker = self._backend
            return
        tracker = engine.get_tracker(self._backend)
        if isinstance(tracker, GeneralTracker) and getattr(tracker, "_blank", False):
            self._logger.info(f"Engine has not initialized {self._backend}. Creating it...")
            try:
                if self._backend not in engine.log_with:
                    engine.log_with.append(self._backend)
                engine.init_trackers("", self._config)
            except Exception as e:
                raise RuntimeError(f"{self.__class__.__name__} can't create tracker: {e}") from e
            tracker = engine.get_tracker(self._backend)
        self._tracker = tracker

    def set(self, attrs: Attributes | None = None) -> None:
        Capsule.set(self, attrs=attrs)
        attrs.tracker = Attributes(scalars=[], images=[])

    def _collect(self, attrs: Attributes) -> None:
        if attrs is None or attrs.tracker is None:
            return
        self._pending_images.extend(attrs.tracker.images or [])
        self._pending_scalars.extend(attrs.tracker.scalars or [])
        attrs.tracker = Attributes(scalars=[], images=[])

    def launch(self, attrs: Attributes | None = None) -> None:
        Capsule.launch(self, attrs=attrs)
        self._collect(attrs)
        self._iters += 1
        if self._iters % self._flush_every == 0:
            self.flush()

    def reset(self, attrs: Attributes | None = None) -> None:
        Capsule.reset(self, attrs=attrs)
        self._collect(attrs)
        self.flush()
        if attrs is not None and "tracker" in attrs:
            del attrs.tracker

    def destroy(self, attrs: Attributes | None = None) -> None:
        self.flush()
        self._tracker = None
        Capsule.destroy(self, attrs=attrs)

    def flush(self) -> None:
        images, scalars = self._pending_images, self._pending_scalars
        self._pending_images, self._pending_scalars = [], []
        if images or scalars:
            self.log(images, scalars)

    def log(self, images: List[Attributes] | None, scalars: List[Attributes] | None) -> None:
        if self._accelerator is None or not self._accelerator.is_main_process or self._tracker is None:
            return
        if images:
            try:
                for image in images:
                    self._tracker.log_images(image.data, step=image.step)
            except Exception as e:
                raise RuntimeError(f"Can't log images: {e}") from e
        if scalars:
            materialize(v for s in scalars for v in s.data.values())
            try:
                for scalar in scalars:
                    self._tracker.log(plain(dict(scalar.data)), step=scalar.step)
            except Exception as e:
                raise RuntimeError(f"Can't log scalars: {e}") from e
