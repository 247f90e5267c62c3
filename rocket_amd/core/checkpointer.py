"""Periodic checkpoint capsule.

Parity (reference ``rocket/core/checkpoint.py``):

* ``Checkpointer(output_dir_format='weights/{:03d}', save_every=None→-1,
  overwrite=True, statefull=True, priority=100)`` (``:59-72``);
* ``setup`` only asserts a project directory exists — it deliberately does *not*
  register itself, so the ``custom_checkpoint_*.pkl`` set matches the reference
  layout (``:74-81``; Appendix C);
* ``launch`` (rank 0): every ``save_every`` Looper iterations — counted globally
  across epochs — writes ``engine.save_state(project_dir/format(iter_idx))``,
  refusing to overwrite when ``overwrite=False`` (``:83-132``);
* state ``{iter_idx: iter_idx + 1}`` (``:134-169``).

Fix: because it is never registered, ``destroy`` is a no-op instead of popping
another capsule's registration and raising (Q1).
"""

from __future__ import annotations

import os

from rocket_amd.core.attributes import Attributes
from rocket_amd.core.capsule import Capsule


class Checkpointer(Capsule):
    def __init__(
        self,
        output_dir_format: str = "weights/{:03d}",
        save_every: int | None = None,
        overwrite: bool = True,
        statefull: bool = True,
        priority: int = 100,
    ) -> None:
        super().__init__(statefull=statefull, priority=priority)
        self._save_every = save_every or -1
        self._output_dir_format = output_dir_format
        self._overwrite = overwrite
        self._iter_idx = 0

    def setup(self, attrs: Attributes | None = None) -> None:
        self.check_accelerator()
        if self._accelerator.project_dir is None:
            raise ValueError(
                "Checkpointer can be used only when project directory is configured. "
                "Current project directory is None. This might be due to the `tag=None` set when creating "
                "`rocket.Launcher`. Set `tag` parameter of `rocket.Launcher` to a specific experiment name"
            )

    def launch(self, attrs: Attributes | None = None) -> None:
        Capsule.launch(self, attrs=attrs)
        if not self._accelerator.is_main_process:
            return
        if self._save_every < 0:
            return
        if (self._iter_idx + 1) % self._save_every == 0:
            out = os.path.join(self._accelerator.project_dir, self._output_dir_format.format(self._iter_idx))
            if not self._overwrite and os.path.exists(out):
                raise RuntimeError(
                    f"{self.__class__.__name__}: Cannot overwrite existing directory. "
                    f"'overwrite' is set to False and '{out}' already exists."
                )
            self._accelerator.save_state(output_dir=out)
            self._logger.info(f"{self.__class__.__name__}: saved {out}")
        self._iter_idx += 1

    def state_dict(self) -> dict:
        return dict(iter_idx=self._iter_idx + 1)

    def load_state_dict(self, state: dict) -> None:
        self._iter_idx = state["iter_idx"]
