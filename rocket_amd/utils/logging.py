"""Rank-aware logging.

Parity: the reference builds every capsule logger with
``accelerate.logging.get_logger`` (``rocket/core/capsule.py:114``), a
``LoggerAdapter`` that emits on the main process only.  This is the same
contract without accelerate: records are dropped on non-zero ranks unless
``main_process_only=False`` is passed per call.
"""

from __future__ import annotations

import logging
import os


def _rank() -> int:
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:  # pragma: no cover - torch always importable here
        pass
    return int(os.environ.get("RANK", "0"))


class RankLogger(logging.LoggerAdapter):
    """Logger adapter that only emits on global rank 0 by default."""

    def log(self, level, msg, *args, main_process_only: bool = True, **kwargs):
        if main_process_only and _rank() != 0:
            return
        if self.isEnabledFor(level):
            msg, kwargs = self.process(msg, kwargs)
            self.logger.log(level, msg, *args, **kwargs)

    def warn(self, msg, *args, **kwargs):  # reference calls .warn (tracker.py:93)
        self.warning(msg, *args, **kwargs)


def get_logger(name: str, level: str | None = None) -> RankLogger:
    logger = logging.getLogger(name)
    lvl = level or os.environ.get("ROCKET_LOG_LEVEL")
    if lvl:
        logger.setLevel(lvl.upper())
    return RankLogger(logger, {})
