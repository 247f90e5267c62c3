"""Deferred device scalars.

The reference reads the loss back to the host on every micro-step
(``loss.item()`` at ``rocket/core/loss.py:97``) and formats it into the progress
bar every iteration (``loop.py:225``) — a device→host synchronisation per step
that, on a GPU, serialises the host with the device.

``LazyScalar`` wraps a 0-d device tensor and behaves like a Python number when
it is *used* (``float()``, formatting, arithmetic, comparisons).  Producers post
``LazyScalar`` objects wherever the reference posted floats; consumers that
print or log them materialise them — batched by :func:`materialize`, which
moves all pending scalars to the host with a single copy.
"""

from __future__ import annotations

import numbers
from typing import Iterable, List

import torch


class LazyScalar(numbers.Real):
    __slots__ = ("_t", "_v", "__weakref__")

    def __init__(self, value):
        if isinstance(value, torch.Tensor):
            self._t = value.detach().reshape(())
            self._v = None
        else:
            self._t = None
            self._v = float(value)

    @property
    def ready(self) -> bool:
        return self._v is not None

    @property
    def tensor(self) -> torch.Tensor | None:
        return self._t

    def value(self) -> float:
        if self._v is None:
            self._v = float(self._t.item())
            self._t = None
        return self._v

    def _set(self, v: float) -> None:
        self._v = float(v)
        self._t = None

    # numbers.Real protocol -------------------------------------------------
    def __float__(self):
        return self.value()

    def __int__(self):
        return int(self.value())

    def __trunc__(self):
        return int(self.value())

    def __floor__(self):
        import math

        return math.floor(self.value())

    def __ceil__(self):
        import math

        return math.ceil(self.value())

    def __round__(self, ndigits=None):
        return round(self.value(), ndigits)

    def __repr__(self):
        return repr(self.value())

    def __str__(self):
        return str(self.value())

    def __format__(self, spec):
        return format(self.value(), spec)

    def __hash__(self):
        return hash(self.value())

    def __eq__(self, o):
        return self.value() == float(o)

    def __lt__(self, o):
        return self.value() < float(o)

    def __le__(self, o):
        return self.value() <= float(o)

    def __add__(self, o):
        return self.value() + float(o)

    __radd__ = __add__

    def __sub__(self, o):
        return self.value() - float(o)

    def __rsub__(self, o):
        return float(o) - self.value()

    def __mul__(self, o):
        return self.value() * float(o)

    __rmul__ = __mul__

    def __truediv__(self, o):
        return self.value() / float(o)

    def __rtruediv__(self, o):
        return float(o) / self.value()

    def __floordiv__(self, o):
        return self.value() // float(o)

    def __rfloordiv__(self, o):
        return float(o) // self.value()

    def __mod__(self, o):
        return self.value() % float(o)

    def __rmod__(self, o):
        return float(o) % self.value()

    def __pow__(self, o):
        return self.value() ** float(o)

    def __rpow__(self, o):
        return float(o) ** self.value()

    def __neg__(self):
        return -self.value()

    def __pos__(self):
        return self.value()

    def __abs__(self):
        return abs(self.value())


def materialize(values: Iterable) -> None:
    """Resolve every pending :class:`LazyScalar` in ``values`` with one D2H copy per device."""
    pending: List[LazyScalar] = [v for v in values if isinstance(v, LazyScalar) and not v.ready]
    if not pending:
        return
    by_dev = {}
    for v in pending:
        by_dev.setdefault(v._t.device, []).append(v)
    for dev, items in by_dev.items():
        host = torch.stack([v._t.float() for v in items]).cpu().tolist()
        for v, x in zip(items, host):
            v._set(x)


def plain(x):
    """Return ``x`` with LazyScalars turned into floats (recursively for dicts/lists)."""
    if isinstance(x, LazyScalar):
        return x.value()
    if isinstance(x, dict):
        return type(x)({k: plain(v) for k, v in x.items()}) if not hasattr(x, "_fields") else x
    if isinstance(x, list):
        return [plain(v) for v in x]
    return x
