"""Structure-preserving maps over nested batches.

Parity: reference ``rocket/utils/collections.py:1-71``.  ``apply_to_collection``
maps ``fn(value, key=k, **kw)`` over the first level of a Mapping or Sequence.
Mutable containers are shallow-copied and updated (so subclasses such as
``Attributes`` or ``OrderedDict`` survive); immutable ones are rebuilt through
their constructor, falling back to a plain dict/list when the type cannot be
rebuilt that way (e.g. namedtuple takes positional fields, handled explicitly).
"""

from __future__ import annotations

import collections.abc as cabc
import copy
from typing import Any, Callable


def is_collection(x: Any) -> bool:
    return isinstance(x, (cabc.Mapping, cabc.Sequence))


def apply_to_mapping(container: cabc.Mapping, fn: Callable, **kwargs):
    mapped = {k: fn(container[k], key=k, **kwargs) for k in container}
    if isinstance(container, cabc.MutableMapping):
        try:
            out = copy.copy(container)
            out.update(mapped)
            return out
        except TypeError:
            return mapped
    try:
        return type(container)(mapped)
    except TypeError:
        return mapped


def apply_to_sequence(container: cabc.Sequence, fn: Callable, **kwargs):
    values = [fn(v, key=i, **kwargs) for i, v in enumerate(container)]
    if isinstance(container, cabc.MutableSequence):
        try:
            out = copy.copy(container)
            out[:] = values
            return out
        except TypeError:
            return values
    if isinstance(container, tuple) and hasattr(container, "_fields"):  # namedtuple
        return type(container)(*values)
    try:
        return type(container)(values)
    except TypeError:
        return values


def apply_to_collection(container, fn: Callable, **kwargs):
    if isinstance(container, cabc.Mapping):
        return apply_to_mapping(container, fn, **kwargs)
    if isinstance(container, cabc.Sequence):
        return apply_to_sequence(container, fn, **kwargs)
    raise TypeError(f"{type(container)} is not a collection.")
