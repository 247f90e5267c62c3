"""Iteration loop over the children of one stage (train or eval).

Parity (reference ``rocket/core/loop.py``):

* ``Looper(capsules, tag, grad_enabled, repeats, run_every, statefull, priority)``
  (``:70-89``), ``repeats=0`` ≡ ``None``; nested loopers rejected (``:265-292``);
* ``set/reset/launch`` only run when ``epoch_idx % run_every == 0`` (``:91-113``);
* ``set`` runs the children first, then infers ``repeats`` = Σ ``_total`` of the
  direct ``Dataset`` children (``:294-323``) and creates ``attrs.looper``
  ``{repeats, state, terminate, tag}`` (``:115-158``);
* each iteration clears ``attrs.batch``, dispatches the children under
  ``torch.set_grad_enabled(grad_enabled)`` and stops on ``looper.terminate``
  (``:182-229``); ``reset`` deletes ``attrs.looper`` (``:160-180``);
* state ``{iter_idx}`` (kept as in the reference, Q3).

Differences: the progress-bar postfix (loss/lr values are device scalars here,
see :mod:`rocket_amd.utils.lazy`) is refreshed at most every ``postfix_interval``
seconds so the host never waits on the device once per step; a resumed epoch
whose datasets are already exhausted is skipped instead of raising (Q4).
"""

from __future__ import annotations

import time

import torch

from rocket_amd.core.attributes import Attributes
from rocket_amd.core.capsule import Capsule
from rocket_amd.core.dispatcher import Dispatcher
from rocket_amd.utils.lazy import materialize


def _green(s: str) -> str:
    return f"\x1b[32m{s}\x1b[0m"


class Looper(Dispatcher):
    def __init__(
        self,
        capsules: list[Capsule],
        tag: str = "Looper",
        grad_enabled: bool = True,
        repeats: int | None = None,
        run_every: int = 1,
        statefull: bool = True,
        priority: int = 1000,
        progress: bool = True,
        postfix_interval: float = 0.5,
    ) -> None:
        super().__init__(capsules=capsules, priority=priority)
        self._statefull = statefull
        self._repeats = None
        self._user_defined_repeats = repeats or None
        self._grad_enabled = grad_enabled
        self._run_every = max(1, int(run_every))
        self._iter_idx = 0
        self._tag = tag
        self._progress = progress
        self._postfix_interval = postfix_interval

    def _active(self, attrs: Attributes | None) -> bool:
        epoch = attrs.launcher.epoch_idx if attrs is not None and attrs.launcher is not None else 0
        return (epoch or 0) % self._run_every == 0

    def set(self, attrs: Attributes | None = None) -> None:
        if not self._active(attrs):
            return
        self._link_deferred_batches()
        Dispatcher.set(self, attrs=attrs)
        self._repeats = self._user_defined_repeats
        if self._repeats is None:
            self.infer_repeats()
        if self._repeats is None:
            raise RuntimeError(
                f"{self.__class__.__name__}: infinite loops are not allowed. Please, specify number of repeats."
            )
        if attrs.looper is None:
            attrs.looper = Attributes(repeats=self._repeats, state=Attributes(), terminate=False, tag=self._tag)

    def _link_deferred_batches(self) -> None:
        """A device-resident Dataset whose batches go straight to a Module whose model gathers its
        own rows (``consumes_pending_rows``, e.g. the fused LeNet step) hands them over deferred:
        the gather then happens inside the model's step kernel (runtime/data.py PendingRows) instead
        of as a launch of its own.  Only for that adjacency in a training loop; everything else
        gets gathered batches."""
        from rocket_amd.core.dataset import Dataset
        from rocket_amd.core.module import Module
        from rocket_amd.runtime.data import DeviceLoader

        caps = self._capsules
        for i, c in enumerate(caps):
            if isinstance(c, Dataset) and isinstance(c._dataloader, DeviceLoader):
                nxt = caps[i + 1] if i + 1 < len(caps) else None
                c._dataloader.defer = bool(self._grad_enabled and isinstance(nxt, Module)
                                           and getattr(nxt, "_gathers_rows", False))

    def reset(self, attrs: Attributes | None = None) -> None:
        if not self._active(attrs):
            return
        Dispatcher.reset(self, attrs=attrs)
        self._repeats = None
        if "looper" in attrs:
            del attrs.looper

    def launch(self, attrs: Attributes | None = None) -> None:
        if not self._active(attrs):
            return
        epoch = attrs.launcher.epoch_idx
        show = bool(self._progress and self._accelerator is not None and self._accelerator.is_local_main_process)
        bar = None
        if show:
            from tqdm import tqdm

            bar = tqdm(total=self._repeats, desc=f"{_green(self._tag)} epoch={epoch}, grad={self._grad_enabled}")
        last = 0.0
        # grad mode entered once for the whole loop and re-established after any iteration whose
        # children switched it outside a context manager: every iteration starts in the mode the
        # reference enters per iteration (loop.py:217), without a context enter/exit per step
        g = self._grad_enabled
        with torch.set_grad_enabled(g):
            for i in range(self._repeats):
                attrs["batch"] = None
                Dispatcher.launch(self, attrs)
                if torch.is_grad_enabled() != g:
                    torch.set_grad_enabled(g)
                if attrs["looper"]["terminate"]:
                    break
                if bar is not None:
                    now = time.monotonic()
                    if now - last >= self._postfix_interval or i == self._repeats - 1:
                        state = attrs.looper.state
                        materialize(v for v in state.values())
                        bar.set_postfix(state, refresh=False)
                        last = now
                    bar.update(1)
        if bar is not None:
            bar.close()
        self._iter_idx = 0
        self._repeats = -1

    def state_dict(self) -> dict:
        return dict(iter_idx=self._iter_idx)

    def load_state_dict(self, state: dict) -> None:
        self._iter_idx = state.get("iter_idx")

    def guard(self, capsules: list[Capsule]) -> None:
        super().guard(capsules)
        for capsule in capsules:
            if isinstance(capsule, Looper):
                raise RuntimeError(f"{self.__class__.__name__}: internal loopers are not allowed.")

    def infer_repeats(self) -> None:
        from rocket_amd.core.dataset import Dataset

        datasets = [c for c in self._capsules if isinstance(c, Dataset)]
        total = sum(d._total for d in datasets)
        if total:
            self._repeats = total
        elif datasets and any(d._resumed_exhausted for d in datasets):
            self._repeats = 0  # epoch finished before the checkpoint was taken (Q4)
        self._logger.info(f"{self.__class__.__name__} infered {self._repeats} repeats.")
