"""Experiment trackers (replaces ``accelerate.tracking`` as used by ``rocket/core/tracker.py``).

The reference's ``Tracker`` capsule resolves a backend name through
``accelerator.get_tracker`` / ``init_trackers`` (``tracker.py:64-105``) and calls
``log(data, step)`` / ``log_images(data, step)`` on rank 0 (``:201-254``).

Backends here:

* ``"jsonl"``  – one JSON object per ``log`` call (always available);
* ``"csv"``    – long-format ``step,key,value`` rows;
* ``"tensorboard"`` – ``torch.utils.tensorboard`` when the ``tensorboard``
  package is importable; otherwise it degrades to ``jsonl`` with a warning
  (tensorboard is not installed in this image; the reference would raise).
* any object exposing ``log(values, step)`` (e.g. an ``accelerate``
  ``GeneralTracker`` instance) can be passed directly.
"""

from __future__ import annotations

import csv
import json
import numbers
import os
import time
from typing import Any, Dict, Optional

from rocket_amd.utils.logging import get_logger

logger = get_logger(__name__)


def _scalar(v: Any) -> Any:
    try:
        import torch

        if isinstance(v, torch.Tensor):
            return v.item() if v.numel() == 1 else v.detach().cpu().tolist()
    except Exception:  # pragma: no cover
        pass
    if hasattr(v, "item") and callable(v.item):
        try:
            return v.item()
        except Exception:
            return v
    return v


class GeneralTracker:
    """Tracker interface.  ``GeneralTracker(_blank=True)`` is the "not initialised" sentinel."""

    name = "general"
    requires_logging_directory = False
    main_process_only = True

    def __init__(self, _blank: bool = False):
        self._blank = _blank

    @property
    def tracker(self):
        return self

    def store_init_configuration(self, values: Dict[str, Any]) -> None:
        return None

    def log(self, values: Dict[str, Any], step: Optional[int] = None, **kwargs) -> None:
        return None

    def log_images(self, values: Dict[str, Any], step: Optional[int] = None, **kwargs) -> None:
        return None

    def finish(self) -> None:
        return None


class JSONLTracker(GeneralTracker):
    name = "jsonl"
    requires_logging_directory = True

    def __init__(self, run_name: str = "", logging_dir: str = "."):
        super().__init__()
        self.dir = os.path.join(logging_dir or ".", run_name) if run_name else (logging_dir or ".")
        os.makedirs(self.dir, exist_ok=True)
        self.path = os.path.join(self.dir, "metrics.jsonl")
        self._fh = open(self.path, "a", buffering=1)

    def store_init_configuration(self, values):
        with open(os.path.join(self.dir, "config.json"), "w") as fh:
            json.dump(values, fh, default=str, indent=2)

    def log(self, values, step=None, **kwargs):
        rec = {"step": step, "time": time.time()}
        rec.update({k: _scalar(v) for k, v in values.items()})
        self._fh.write(json.dumps(rec, default=str) + "\n")

    def log_images(self, values, step=None, **kwargs):
        d = os.path.join(self.dir, "images")
        os.makedirs(d, exist_ok=True)
        try:
            import torch

            for k, v in values.items():
                torch.save(v, os.path.join(d, f"{k.replace('/', '_')}_{step}.pt"))
        except Exception as e:  # pragma: no cover
            logger.warning(f"jsonl tracker could not store images: {e}")

    def finish(self):
        if not self._fh.closed:
            self._fh.close()


class CSVTracker(GeneralTracker):
    name = "csv"
    requires_logging_directory = True

    def __init__(self, run_name: str = "", logging_dir: str = "."):
        super().__init__()
        self.dir = os.path.join(logging_dir or ".", run_name) if run_name else (logging_dir or ".")
        os.makedirs(self.dir, exist_ok=True)
        self.path = os.path.join(self.dir, "metrics.csv")
        new = not os.path.exists(self.path)
        self._fh = open(self.path, "a", newline="", buffering=1)
        self._w = csv.writer(self._fh)
        if new:
            self._w.writerow(["step", "key", "value"])

    def log(self, values, step=None, **kwargs):
        for k, v in values.items():
            v = _scalar(v)
            if isinstance(v, numbers.Number):
                self._w.writerow([step, k, v])

    def finish(self):
        if not self._fh.closed:
            self._fh.close()


class TensorBoardTracker(GeneralTracker):
    name = "tensorboard"
    requires_logging_directory = True

    def __init__(self, run_name: str = "", logging_dir: str = "."):
        super().__init__()
        from torch.utils.tensorboard import SummaryWriter  # needs the `tensorboard` package

        self.writer = SummaryWriter(os.path.join(logging_dir or ".", run_name))

    @property
    def tracker(self):
        return self.writer

    def store_init_configuration(self, values):
        self.writer.add_hparams({k: v for k, v in values.items() if isinstance(v, (int, float, str, bool))}, {})

    def log(self, values, step=None, **kwargs):
        for k, v in values.items():
            v = _scalar(v)
            if isinstance(v, numbers.Number):
                self.writer.add_scalar(k, v, global_step=step)
            elif isinstance(v, str):
                self.writer.add_text(k, v, global_step=step)
        self.writer.flush()

    def log_images(self, values, step=None, **kwargs):
        for k, v in values.items():
            self.writer.add_images(k, v, global_step=step, dataformats=kwargs.get("dataformats", "NCHW"))
        self.writer.flush()

    def finish(self):
        self.writer.close()


TRACKERS = {"jsonl": JSONLTracker, "csv": CSVTracker, "tensorboard": TensorBoardTracker}


def make_tracker(name: str, run_name: str, logging_dir: str) -> GeneralTracker:
    cls = TRACKERS.get(name)
    if cls is None:
        raise ValueError(f"unknown tracker backend {name!r}; known: {sorted(TRACKERS)}")
    try:
        return cls(run_name, logging_dir)
    except ImportError as e:
        logger.warning(f"tracker '{name}' unavailable ({e}); falling back to jsonl")
        t = JSONLTracker(run_name, logging_dir)
        t.name = name  # resolvable under the requested name
        return t
